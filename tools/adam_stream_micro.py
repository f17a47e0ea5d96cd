"""Dense Adam step (optim.hip::adam_kernel through pv_adam_dev) at the MLP (16 M) and BERT
(110 M) parameter counts: plain vs non-temporal streams, workgroup caps; interleaved rounds,
CUDA-event timed; effective HBM rate at 28 B / parameter.

    python tools/adam_stream_micro.py [--n 16e6,110e6] [--rounds 5]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", default="16e6,110e6")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from dnn_page_vectors_amd.ops._common import lib, P, stream
    L = lib()
    dev = torch.device("cuda")
    arms = [4096, 16384]
    out = {}
    for n in [int(float(x)) for x in a.n.split(",")]:
        p, g, m, v = (torch.randn(n, device=dev) * 0.01 for _ in range(4))
        v.abs_()
        t = torch.zeros(2, device=dev)  # {step, warmup steps}
        s = stream(dev)
        res = {arm: [] for arm in arms}
        for _ in range(a.rounds):
            for cap in arms:
                L.pv_adam_set_grid(cap)
                for _ in range(3):
                    L.pv_adam_dev(P(p), P(g), P(m), P(v), n, P(t), 1e-4, 0.9, 0.999, 1e-7, 0.0, 0, None, s)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    L.pv_adam_dev(P(p), P(g), P(m), P(v), n, P(t), 1e-4, 0.9, 0.999, 1e-7, 0.0, 0, None, s)
                e1.record()
                torch.cuda.synchronize()
                res[cap].append(e0.elapsed_time(e1) / a.iters * 1e3)
        for cap, xs in res.items():
            us = statistics.median(xs)
            out[f"n{n}_cap{cap}"] = {"us": round(us, 1), "TBps": round(28 * n / us / 1e6, 2)}
    L.pv_adam_set_grid(16384)  # the default
    print(json.dumps(out))


if __name__ == "__main__":
    main()
