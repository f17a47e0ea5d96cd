"""Build variant HIP libraries that differ only in compile-time macros of one kernel source
(e.g. the conv forward chunk size PV_CONV_R), for same-box A/B runs selected with
PAGEVEC_HIP_LIB=<path>:

    python tools/conv_variant_build.py --src conv_pool_fwd.hip --define PV_CONV_R=96 PV_CONV_R=128
    -> dnn_page_vectors_amd/lib/variants/libpagevec_hip_PV_CONV_R_96.so, ...
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dnn_page_vectors_amd import _build as B  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--src", nargs="+", default=["conv_pool_fwd.hip"],
                    help="sources compiled with the define (e.g. every user of a common.h switch)")
    ap.add_argument("--define", nargs="+", required=True)
    a = ap.parse_args()
    B.build_hip()  # the release objects of every other source
    kdir = os.path.join(B.CSRC, "kernels")
    srcs = B._sources(kdir, ".hip")
    hdrs = B._headers(kdir)
    base = []
    for s in srcs:
        key = B._digest([s] + hdrs, list(B.HIP_FLAGS) + [B.HIPCC])
        base.append((s, os.path.join(B.OBJ, f"hip_{os.path.splitext(os.path.basename(s))[0]}_{key}.o")))
    vdir = os.path.join(B.LIB, "variants")
    os.makedirs(vdir, exist_ok=True)
    for d in a.define:
        tag = d.replace("=", "_")
        vobj = {}
        for sname in a.src:
            obj = os.path.join(vdir, f"{tag}_{os.path.splitext(sname)[0]}.o")
            B._run([B.HIPCC] + list(B.HIP_FLAGS) + [f"-D{d}", "-I", kdir, "-c", os.path.join(kdir, sname), "-o", obj],
                   True)
            vobj[sname] = obj
        objs = [vobj.get(os.path.basename(s), o) for s, o in base]
        out = os.path.join(vdir, f"libpagevec_hip_{tag}.so")
        B._run([B.HIPCC, f"--offload-arch={B.ARCH}", "-fPIC", "-shared", "-o", out] + objs, True)
        print(out)


if __name__ == "__main__":
    main()
