// Stable LSD radix sort of (uint32 key, uint32 value) pairs on the device (rocPRIM via hipCUB).
// Used to bucket sparse-gradient entries by destination row (deterministic order within
// a bucket = emission order, so the segment sums are reproducible run to run).
#include <hipcub/hipcub.hpp>
#include <rocprim/rocprim.hpp>
#include "common.h"

PV_API long pv_sort_pairs_temp_bytes(long n, int end_bit) {
  size_t bytes = 0;
  hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const unsigned*)nullptr, (unsigned*)nullptr,
                                     (const unsigned*)nullptr, (unsigned*)nullptr, (int)n, 0, end_bit);
  return (long)bytes;
}

PV_API int pv_sort_pairs_u32(void* temp, long temp_bytes, const unsigned* keys_in, unsigned* keys_out,
                             const unsigned* vals_in, unsigned* vals_out, long n, int end_bit, void* stream) {
  size_t bytes = (size_t)temp_bytes;
  hipError_t e = hipcub::DeviceRadixSort::SortPairs(temp, bytes, keys_in, keys_out, vals_in, vals_out, (int)n, 0,
                                                    end_bit, (hipStream_t)stream);
  return (int)e;
}

// Same stable sort with the values being the input positions 0..n-1 (a rocPRIM counting
// iterator): the conv backward's emitted value of entry i is i itself, so the emit kernel
// need not write (and the first sort pass need not read) an n-entry value array.
PV_API long pv_sort_iota_temp_bytes(long n, int end_bit) {
  size_t bytes = 0;
  rocprim::radix_sort_pairs(nullptr, bytes, (const unsigned*)nullptr, (unsigned*)nullptr,
                            rocprim::counting_iterator<unsigned>(0u), (unsigned*)nullptr, (size_t)n, 0u,
                            (unsigned)end_bit);
  return (long)bytes;
}

PV_API int pv_sort_iota_u32(void* temp, long temp_bytes, const unsigned* keys_in, unsigned* keys_out,
                            unsigned* vals_out, long n, int end_bit, void* stream) {
  size_t bytes = (size_t)temp_bytes;
  hipError_t e = rocprim::radix_sort_pairs(temp, bytes, keys_in, keys_out, rocprim::counting_iterator<unsigned>(0u),
                                           vals_out, (size_t)n, 0u, (unsigned)end_bit, (hipStream_t)stream);
  return (int)e;
}

// 2-byte keys (token ids < 65535), values = input positions (counting iterator)
PV_API long pv_sort_iota_u16_temp_bytes(long n, int end_bit) {
  size_t bytes = 0;
  rocprim::radix_sort_pairs(nullptr, bytes, (const unsigned short*)nullptr, (unsigned short*)nullptr,
                            rocprim::counting_iterator<unsigned>(0u), (unsigned*)nullptr, (size_t)n, 0u,
                            (unsigned)end_bit);
  return (long)bytes;
}

PV_API int pv_sort_iota_u16(void* temp, long temp_bytes, const void* keys_in, void* keys_out, unsigned* vals_out,
                            long n, int end_bit, void* stream) {
  size_t bytes = (size_t)temp_bytes;
  hipError_t e = rocprim::radix_sort_pairs(temp, bytes, (const unsigned short*)keys_in, (unsigned short*)keys_out,
                                           rocprim::counting_iterator<unsigned>(0u), vals_out, (size_t)n, 0u,
                                           (unsigned)end_bit, (hipStream_t)stream);
  return (int)e;
}
