"""Runtime knobs outside ``Configuration``: what a run actually had in effect.

The model, data, loss and optimizer live in ``config.Configuration``.  What is
left to the environment is of three kinds, listed here with their production default so a
record can say which of them a run changed:

* ``ab``       — same-process A/B arms of measured engineering choices (docs/PERF.md has the
                 numbers); the default is the measured winner, the other arm stays for re-runs
                 on new hardware or ROCm releases;
* ``runtime``  — process plumbing (library selection, tracing, fault injection, launch);
* ``hip``      — HIP / HSA runtime variables the step's performance depends on.

``in_effect()`` is written into every ``bench.py`` record (``runtime_knobs``): a run with a
stray knob is visible as such.
"""
from __future__ import annotations

import os
from typing import Dict

# name -> (kind, production default, what it selects)
KNOBS: Dict[str, tuple] = {
    # conv tower (ops/conv_pool.py, conv_pool_fwd.hip / conv_pool_bwd.hip / radix_sort.hip)
    "PAGEVEC_CONV_DBG": ("ab", "0", "conv forward variant / timing ablation (0 = v7 production)"),
    "PAGEVEC_REDUCE_EPW": ("ab", "512", "sorted dTable entries per wave in reduce7"),
    "PAGEVEC_R7_OCC": ("ab", "8", "reduce7 register cap (waves per SIMD)"),
    "PAGEVEC_DW_STREAM": ("ab", "0", "page-tower dW on a side stream"),
    "PAGEVEC_BIAS_SINK": ("ab", "1", "conv bias gradients written by the dW kernel"),
    "PAGEVEC_SIDE_PER_STREAM": ("ab", "1", "one side stream per calling stream"),
    "PAGEVEC_FWD_EMIT": ("ab", "1", "dTable sort keys emitted by the forward's loader waves"),
    "PAGEVEC_EARLY_SORT": ("ab", "1", "dTable key sort right after the forward, side stream"),
    "PAGEVEC_EARLY_SORT_SKIP": ("ab", "1", "no early sort for 128 < L < 1024"),
    "PAGEVEC_RSORT_IPT": ("ab", "auto", "radix sort items per thread"),
    "PAGEVEC_F32_NATIVE": ("ab", "1", "fp32 (reference precision) conv on the fp32-MFMA kernels"),
    "PAGEVEC_F32_DX_LDS": ("ab", "1", "fp32 dTable in LDS tables for small vocabularies"),
    "PAGEVEC_F32_MASK": ("ab", "1", "fp32 forward dropout keep-bit plane"),
    # bags, dense, loss, optimizer
    "PAGEVEC_BAG_SPARSE_BWD": ("ab", "1", "short-bag backward by sorted token runs"),
    "PAGEVEC_BAG_EPW": ("ab", "64", "sorted entries per wave of the short-bag backward"),
    "PAGEVEC_BAG_SPLITK": ("ab", "0", "vocabulary split of the counts GEMM (0 = auto)"),
    "PAGEVEC_COLSUM": ("ab", "1", "column sums on the HIP kernel (0: torch reductions)"),
    "PAGEVEC_WGRAD_WG": ("ab", "512", "dense-layer weight-gradient workgroup target"),
    "PAGEVEC_QUERY_STREAM": ("ab", "1", "query tower on its own stream beside the page tower"),
    "PAGEVEC_BAG_COUNTS16": ("ab", "1", "16-bit packed LDS counts histogram"),
    "PAGEVEC_BAG_GEMM": ("ab", "auto", "long-bag GEMMs on the count matrix: in-tree bagd_mm_kernel (dense) or "
                                         "hipBLASLt (lib); auto = dense eager, lib inside a graph capture"),
    "PAGEVEC_FP8_BAG": ("ab", "1", "fp8 towers: page bag on the MX fp8 MFMA"),
    "PAGEVEC_FP8_BWD": ("ab", "0", "fp8 towers: bag weight gradient on the MX fp8 MFMA (e4m3 counts^T x e4m3 G)"),
    "PAGEVEC_DENSE_BWD": ("ab", "hip", "dense-layer backward on HIP kernels or the library"),
    "PAGEVEC_DIRECT_GRAD": ("ab", "1", "kernels write the flat gradient buffer directly"),
    "PAGEVEC_RESID_FUSE": ("ab", "1", "BERT residual gradients fused into dX GEMMs"),
    "PAGEVEC_CONV_SHORT": ("ab", "1", "conv forward: one 48-row chunk for sequences up to 50 tokens (query tower)"),
    "PAGEVEC_ATTN_BGRAD": ("ab", "1", "qkv bias gradient from the attention backward's partial column sums"),
    "PAGEVEC_BERT_EMBED": ("ab", "1", "BERT embedding front end as one fused gather + add kernel"),
    "PAGEVEC_CAPTURE_STREAMS": ("ab", "1", "hipGraph captures keep the query-tower / early-sort side streams"),
    "PAGEVEC_STEP_PRIORITY": ("ab", "1", "eager step on a high-priority stream (query tower / side streams normal)"),
    "PAGEVEC_NO_MIRROR": ("ab", "0", "no bf16 mirror written by the Adam kernel"),
    # process plumbing
    "PAGEVEC_HIP_LIB": ("runtime", "", "path of the kernel library to load"),
    "PAGEVEC_DEBUG_KERNELS": ("runtime", "0", "load the PV_CHECK debug kernel library"),
    "PAGEVEC_NO_AUTOBUILD": ("runtime", "0", "never build the native libraries on import"),
    "PAGEVEC_ARCH": ("runtime", "gfx950", "offload arch of the build"),
    "PAGEVEC_BACKEND": ("runtime", "auto", "hip kernels or eager torch ops"),
    "PAGEVEC_ROCTX": ("runtime", "0", "roctx ranges around the step phases"),
    "PAGEVEC_FAULT_STEP": ("runtime", "-1", "raise at this step (resume tests)"),
    "PAGEVEC_FORCE_DIST": ("runtime", "0", "force the collective paths on a world-1 group (tests)"),
    "PAGEVEC_DIST_BACKEND": ("runtime", "", "process-group backend override (gloo rehearsal)"),
    # HIP / HSA runtime
    "GPU_MAX_HW_QUEUES": ("hip", "4", "hardware queues per process (HIP default 4)"),
    "HSA_ENABLE_IPC_MODE_LEGACY": ("hip", "0", "dmabuf IPC for RCCL on this driver"),
}


def in_effect() -> Dict[str, str]:
    """Every PAGEVEC_* variable set in this process's environment (registered or not) and the
    value in effect of every ``hip`` knob (``<default> (unset)`` when the runtime's default
    applies)."""
    out = {k: v for k, v in sorted(os.environ.items()) if k.startswith("PAGEVEC_")}
    for k, (kind, default, _) in KNOBS.items():
        if kind == "hip":
            out[k] = os.environ.get(k, f"{default} (unset)")
    return out


def non_default() -> Dict[str, str]:
    """The registered knobs whose environment value differs from the production default."""
    return {k: os.environ[k] for k, (_, d, _) in KNOBS.items() if k in os.environ and os.environ[k] != d}
