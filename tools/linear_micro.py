"""Every BERT linear GEMM (config 4, T = 73728 tokens) per call: torch (bundled hipBLASLt
heuristic) vs lt_gemm.hip heuristic #1 vs lt_gemm.hip with the top-16 candidates timed
(PAGEVEC_LT_TUNE).  Uniform random operands (constant ones draw less power, clock higher
and overstate the rate by ~40 % on this chip: profiles/r5_lt/lt_shapes.log)."""
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
    for name, K, N in (("qkv", H, 3 * H), ("o", H, H), ("ffn1", H, I), ("ffn2", I, H)):
        x, w, dy = rnd(T, K), rnd(N, K), rnd(T, N)
        y = torch.empty(T, N, dtype=torch.bfloat16, device=dev)
        dx = torch.empty(T, K, dtype=torch.bfloat16, device=dev)
        r = {"fwd_torch": ev(lambda: x @ w.t()), "dx_torch": ev(lambda: dy @ w)}
        for tune in (False, True):
            tops.LT_TUNE = tune
            tops._LT_TUNE_SET[0] = None
            tag = "tuned" if tune else "h1"
            r[f"fwd_lt_{tag}"] = ev(lambda: tops.lt_mm(x, w, y, tb=True))
            r[f"dx_lt_{tag}"] = ev(lambda: tops.lt_mm(dy, w, dx))
            r[f"dxres_lt_{tag}"] = ev(lambda: tops.lt_mm(dy, w, dx, beta=1.0))
        r["dxres_torch"] = ev(lambda: dx.addmm_(dy, w))
        res[name] = r
        print(name, json.dumps(r), flush=True)
    tops.LT_TUNE = False
    tot = {k: round(sum(v[k] for v in res.values()), 1) for k in next(iter(res.values()))}
    print("sum", json.dumps(tot), flush=True)


if __name__ == "__main__":
    main()
