"""The MLP / chunked page-bag GEMMs (dense bf16 counts x table, C^T x dZ) on torch's calls
(split-K bmm + colsum, mm) vs lt_gemm.hip heuristic #1 and with the top-16 candidates timed.
Random operands; counts from the bench's synthetic Zipf pages."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def ev(fn, it=20):
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
    from dnn_page_vectors_amd.config import Configuration
    from dnn_page_vectors_amd.data.synthetic import SyntheticPairs, spec_from_config
    from dnn_page_vectors_amd.ops import embedding as eops
    from dnn_page_vectors_amd.ops import transformer as tops

    dev = torch.device("cuda")
    N, L, V, E = 4096, 2000, 30000, 512
    cfg = Configuration(feature_level="ngram", vocab_hash_size=V, query_length=45, document_length=L, J=0)
    data = SyntheticPairs(spec_from_config(cfg, V, num_pages=N), dev, seed=5)
    ids = data.pages[:N].contiguous()
    C, lens = eops._counts(ids, V, 0)
    Cv = C[:, :V]
    W16 = ((torch.rand(V, E, device=dev) * 2 - 1) * 0.05).bfloat16()
    gs = (torch.rand(N, E, device=dev) * 2 - 1).bfloat16()
    r = {"fwd_torch_splitk": ev(lambda: eops._counts_gemm(Cv, W16))}
    out = torch.empty(V, E, device=dev)
    r["wgrad_torch"] = ev(lambda: torch.mm(Cv.t(), gs, out_dtype=torch.float32, out=out))
    yf = torch.empty(N, E, device=dev)
    for tune in (False, True):
        tops.LT_TUNE = tune
        tops._LT_TUNE_SET[0] = None
        t = "tuned" if tune else "h1"
        r[f"fwd_lt_{t}"] = ev(lambda: tops.lt_mm(Cv, W16, yf))            # fp32 out, no split
        r[f"wgrad_lt_{t}"] = ev(lambda: tops.lt_mm(Cv, gs, out, ta=True))
    tops.LT_TUNE = False
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
