"""The BERT GEMM shapes of tools/native/lt_shapes.cpp through torch (its bundled hipBLASLt), for
the side-by-side with the system ROCm's hipBLASLt."""
import torch


def ev(fn, it=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / it


def main():
    dev = torch.device("cuda")
    T = 73728
    bf = torch.bfloat16
    cases = [("qkv_fwd  T x 2304 x 768", (T, 768), (2304, 768), "nt", False),
             ("ffn1_fwd T x 3072 x 768", (T, 768), (3072, 768), "nt", False),
             ("ffn2_fwd T x 768 x 3072", (T, 3072), (768, 3072), "nt", False),
             ("ffn2_dx  T x 3072 x 768", (T, 768), (768, 3072), "nn", False),
             ("ffn1_dw  3072 x 768 x T (fp32)", (T, 3072), (T, 768), "tn", True),
             ("square 8192", (8192, 8192), (8192, 8192), "nt", False)]
    for name, sa, sb, mode, f32 in cases:
        a = (torch.rand(*sa, device=dev) * 2 - 1).to(bf)  # uniform [-1, 1) as the C++ tool
        b = (torch.rand(*sb, device=dev) * 2 - 1).to(bf)
        if mode == "nt":
            fn = lambda: a @ b.t()  # noqa: E731
            fl = 2.0 * sa[0] * sa[1] * sb[0]
        elif mode == "nn":
            fn = lambda: a @ b  # noqa: E731
            fl = 2.0 * sa[0] * sa[1] * sb[1]
        else:
            fn = lambda: torch.mm(a.t(), b, out_dtype=torch.float32)  # noqa: E731
            fl = 2.0 * sa[1] * sa[0] * sb[1]
        ms = ev(fn)
        print(f"{name:32s} torch {ms:.3f} ms ({fl / ms / 1e9:.0f} TF/s)", flush=True)


if __name__ == "__main__":
    main()
