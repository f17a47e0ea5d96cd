"""BERT weight gradients (fp32 dW = dY^T X over T = 73728 tokens): the split-K batched GEMM +
fixed-order column sum (ops/transformer.py::wgrad_f32) at token splits 1 / 4 / 8 / 16 (first run) and 16 / 32 / 64."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


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
    return round(a.elapsed_time(b) / it * 1000, 1)


def main():
    from dnn_page_vectors_amd.ops import transformer as tops

    dev = torch.device("cuda")
    T, H, I = 73728, 768, 3072
    rnd = lambda *s: (torch.rand(*s, device=dev) * 2 - 1).bfloat16()  # noqa: E731
    res = {}
    orig = tops._wgrad_splits
    for name, N, K in (("qkv", 3 * H, H), ("o", H, H), ("ffn1", I, H), ("ffn2", H, I)):
        dy, x = rnd(T, N), rnd(T, K)
        out = torch.empty(N, K, device=dev)
        r = {}
        for sk in (16, 32, 64):
            tops._wgrad_splits = lambda T_, sk=sk: sk
            r[f"sk{sk}"] = ev(lambda: tops.wgrad_f32(dy, x, out=out))
        res[name] = r
        print(name, json.dumps(r), flush=True)
    tops._wgrad_splits = orig
    print("sum", json.dumps({k: round(sum(v[k] for v in res.values()), 1) for k in ("sk16", "sk32", "sk64")}))


if __name__ == "__main__":
    main()
