// Host-side sanitizer driver for the C++ runtime (CPU ASan/UBSan build of the
// featurizer).  Linked directly against csrc/runtime/featurize.cpp and built with
// -fsanitize=address,undefined by tests/test_sanitizers.py; exercises every C entry point
// on random bytes (invalid UTF-8, huge tokens), all feature modes with a vocabulary and
// with hashing, several thread counts, and a JSONL file full of malformed records
// (truncated strings, bad escapes, lone surrogates, wrong negative counts).
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

extern "C" {
void* pv_vocab_new();
void pv_vocab_free(void*);
void pv_vocab_add(void*, const char*, int32_t);
int64_t pv_vocab_size(void*);
int pv_featurize(const char**, int, int, int, void*, int, int, int, int32_t*, int);
int64_t pv_clean_str(const char*, char*, int64_t);
void* pv_dataset_open(const char*, int, int);
int64_t pv_dataset_size(void*);
int64_t pv_dataset_skipped(void*);
void pv_dataset_close(void*);
int pv_dataset_batch(void*, const int64_t*, int, int, int, int, void*, int, int, int, int32_t*, int32_t*, int);
int64_t pv_dataset_row_text(void*, int64_t, int, char*, int64_t);
}

static uint64_t g_state = 0x9E3779B97F4A7C15ull;
static uint32_t rnd() {
  g_state ^= g_state << 13;
  g_state ^= g_state >> 7;
  g_state ^= g_state << 17;
  return (uint32_t)g_state;
}

static std::string random_text(int maxlen) {
  static const char* pieces[] = {"statue", " ", "of", "liberty", "!", "Mütze", "€", "ß", "#1", "$25.00", "a-b_c",
                                 "\xff", "\xc3", "\xe2\x82", "\xf0\x9f\x98\x80", "\t", "\n", "..", "ÄÖÜ", "x"};
  std::string s;
  const int n = (int)(rnd() % (unsigned)maxlen);
  while ((int)s.size() < n) {
    if (rnd() % 4 == 0) s.push_back((char)(1 + rnd() % 255));
    else s += pieces[rnd() % (sizeof(pieces) / sizeof(pieces[0]))];
  }
  return s;
}

static std::string json_escape(const std::string& x) {
  std::string o;
  for (unsigned char c : x) {
    if (c == '"' || c == '\\') {
      o.push_back('\\');
      o.push_back((char)c);
    } else if (c < 0x20) {
      char t[8];
      snprintf(t, sizeof t, "\\u%04x", c);
      o += t;
    } else {
      o.push_back((char)c);
    }
  }
  return o;
}

int main(int argc, char** argv) {
  const char* tmp = argc > 1 ? argv[1] : "/tmp/pv_fuzz.jsonl";
  const int iters = argc > 2 ? atoi(argv[2]) : 300;
  void* voc = pv_vocab_new();
  const char* toks[] = {"<PAD/>", "<UNK/>", " ", "sta", "tat", "statue", "of", "s", "t", "a"};
  for (int i = 0; i < 10; ++i) pv_vocab_add(voc, toks[i], i);
  if (pv_vocab_size(voc) != 10) return 10;

  char buf[256];
  for (int it = 0; it < iters; ++it) {
    const std::string s = random_text(400);
    if (pv_clean_str(s.c_str(), buf, (int64_t)(rnd() % sizeof(buf))) < 0) return 11;
    std::vector<std::string> texts(1 + rnd() % 17);
    std::vector<const char*> ptrs;
    for (auto& t : texts) {
      t = random_text(300);
      ptrs.push_back(t.c_str());
    }
    for (int mode = 0; mode < 3; ++mode) {
      const int len = 1 + (int)(rnd() % 64);
      std::vector<int32_t> out(texts.size() * (size_t)len, -7);
      const int threads = 1 + (int)(rnd() % 4);
      if (pv_featurize(ptrs.data(), (int)ptrs.size(), mode, len, voc, 0, 1, 0, out.data(), threads) != 0) return 12;
      for (int32_t v : out)
        if (v < 0 || v > 9) return 13;
      const int V = 2 + (int)(rnd() % 5000);
      if (pv_featurize(ptrs.data(), (int)ptrs.size(), mode, len, nullptr, V, 1, 0, out.data(), threads) != 0)
        return 14;
      for (int32_t v : out)
        if (v < 0 || v >= V) return 15;
    }
  }

  FILE* f = fopen(tmp, "w");
  if (!f) return 20;
  const char* bad[] = {"{\"q\": \"x\", \"doc_corr\": \"y\", \"doc_incorr\": [\"a\", \"b\"]}",
                       "{\"q\": \"trunc",
                       "{\"q\": \"\\ud800\", \"doc_corr\": \"\\u00fc\", \"doc_incorr\": [\"1\",\"2\",\"3\"]}",
                       "not json",
                       "{\"q\": \"a\\\"b\\\\c\\n\", \"doc_corr\": \"p\", \"doc_incorr\": [\"\",\"\",\"\"]}",
                       "{}",
                       "[1,2,3]",
                       "{\"q\": 5, \"doc_corr\": null, \"doc_incorr\": {}}"};
  int good = 0;
  for (int i = 0; i < 200; ++i) {
    if (rnd() % 3 == 0) {
      fputs(bad[rnd() % 8], f);
      fputc('\n', f);
      continue;
    }
    fprintf(f, "{\"q\": \"%s\", \"doc_corr\": \"%s\", \"doc_incorr\": [\"%s\", \"%s\", \"%s\"]}\n",
            json_escape(random_text(40)).c_str(), json_escape(random_text(200)).c_str(),
            json_escape(random_text(50)).c_str(), json_escape(random_text(50)).c_str(),
            json_escape(random_text(50)).c_str());
    ++good;
  }
  fclose(f);
  void* ds = pv_dataset_open(tmp, 3, 3);
  if (!ds) return 21;
  const int64_t n = pv_dataset_size(ds);
  if (n < good) return 22;
  std::vector<int64_t> rows;
  for (int64_t r = 0; r < n; ++r) rows.push_back((r * 7) % n);
  for (int mode = 0; mode < 3; ++mode) {
    std::vector<int32_t> q(rows.size() * 9), d(rows.size() * 4 * 33);
    if (pv_dataset_batch(ds, rows.data(), (int)rows.size(), mode, 9, 33, mode == 1 ? nullptr : voc,
                         mode == 1 ? 1000 : 0, 1, 0, q.data(), d.data(), 4) != 0)
      return 23;
  }
  int64_t bad_row = n + 5;
  std::vector<int32_t> q1(9), d1(4 * 33);
  if (pv_dataset_batch(ds, &bad_row, 1, 0, 9, 33, voc, 0, 1, 0, q1.data(), d1.data(), 1) == 0) return 24;
  for (int64_t r = 0; r < n; ++r)
    for (int field = 0; field < 6; ++field) pv_dataset_row_text(ds, r, field, buf, (int64_t)(rnd() % sizeof(buf)));
  pv_dataset_close(ds);
  pv_vocab_free(voc);
  printf("ok rows=%lld\n", (long long)n);
  return 0;
}
