"""Which hipBLASLt epilogues (lt_gemm.hip) have solutions for the BERT FFN shapes on this box:
prints the launcher status per (epilogue, bias dtype, aux type attribute, output dtype)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    from dnn_page_vectors_amd.ops import transformer as tops

    dev = torch.device("cuda")
    T, H, I = 4096, 768, 3072
    x = torch.randn(T, H, device=dev).bfloat16()
    w1 = torch.randn(I, H, device=dev).bfloat16()
    w2 = torch.randn(H, I, device=dev).bfloat16()
    dy = torch.randn(T, H, device=dev).bfloat16()
    for odt in (torch.bfloat16, torch.float32):
        for bias_dt in (torch.float32, torch.bfloat16):
            b = torch.zeros(I, dtype=bias_dt, device=dev)
            for epi in (2, 3, 4, 5, 6, 7, 102, 103, 104, 107):
                out = torch.empty(T, I, dtype=odt, device=dev)
                aux = torch.empty(T, I, dtype=torch.bfloat16, device=dev)
                fwd = epi % 100 in (2, 5, 6, 7)
                biased = epi % 100 in (2, 4, 6)
                auxed = epi % 100 in (2, 3, 4, 7)
                if fwd:
                    r = tops.lt_mm(x, w1, out, tb=True, epi=epi, bias=b if biased else None, aux=aux if auxed else None)
                else:
                    r = tops.lt_mm(dy, w2, out, epi=epi, bias=b if biased else None, aux=aux)
                torch.cuda.synchronize()
                print(f"out {odt} epi {epi} bias {bias_dt}: status {r}", flush=True)


if __name__ == "__main__":
    main()
