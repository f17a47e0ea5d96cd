"""Same-process A/B of a trainer-level module flag on the headline step (interleaved rounds,
CUDA-event timed), e.g. the query-tower-first forward order:

    python tools/step_flag_ab.py --module dnn_page_vectors_amd.ops.conv_pool --flag DW_SIDE_STREAM
"""
import argparse
import importlib
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--module", default="dnn_page_vectors_amd.train.trainer")
    ap.add_argument("--flag", default="DW_SIDE_STREAM")
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--steps", type=int, default=15)
    ap.add_argument("--vals", default="0,1", help="the two values A/B'd (Python literals); 0/1 -> False/True")
    ap.add_argument("--preset", default="cdssm_ngram_bf16")
    ap.add_argument("--set", action="append", default=[], metavar="KEY=VALUE")
    ap.add_argument("--setter", default="", help="a libpagevec_hip setter (e.g. pv_conv_r7_set_occ) instead of a flag")
    ap.add_argument("--env", default="", help="an environment variable read at call time (e.g. PAGEVEC_QUERY_STREAM): "
                                              "the two values are its string values")
    a = ap.parse_args()
    from dnn_page_vectors_amd.config import preset_config
    from dnn_page_vectors_amd.data.synthetic import SyntheticPairs, spec_from_config
    from dnn_page_vectors_amd.models import build_model
    from dnn_page_vectors_amd.parallel import dist as pdist
    from dnn_page_vectors_amd.train.trainer import Trainer

    info = pdist.init_distributed()
    cfg = preset_config(a.preset)
    if a.set:
        cfg = cfg.override(a.set)
    V = cfg.vocab_hash_size
    dev = info.device
    tr = Trainer(cfg, build_model(cfg, V), dev, graph=False)
    data = SyntheticPairs(spec_from_config(cfg, V, num_pages=65536), dev, seed=1337)
    pool = [data.batch(cfg.batch_size) for _ in range(4)]
    import ast

    mod = importlib.import_module(a.module)
    va, vb = (ast.literal_eval(v) for v in a.vals.split(","))
    if a.vals == "0,1" and not a.setter and not a.env:
        va, vb = False, True
    from dnn_page_vectors_amd.ops._common import lib

    def setv(v):
        if a.env:
            os.environ[a.env] = str(v)
        elif a.setter:
            getattr(lib(), a.setter)(int(v))
        else:
            setattr(mod, a.flag, v)
    for i in range(5):
        tr.train_step(*pool[i % 4])
    res = {va: [], vb: []}
    k = 0
    for r in range(a.rounds):
        for val in ((va, vb) if r % 2 == 0 else (vb, va)):
            setv(val)
            tr.train_step(*pool[k % 4])
            k += 1
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.steps):
                tr.train_step(*pool[k % 4])
                k += 1
            e1.record()
            torch.cuda.synchronize()
            res[val].append(e0.elapsed_time(e1) / a.steps)
    print(json.dumps({"preset": a.preset, "flag": a.env or a.setter or a.flag, "a": str(va), "b": str(vb),
                      "a_ms": [round(x, 3) for x in res[va]], "b_ms": [round(x, 3) for x in res[vb]],
                      "a_median": round(statistics.median(res[va]), 3),
                      "b_median": round(statistics.median(res[vb]), 3)}), flush=True)


if __name__ == "__main__":
    main()
