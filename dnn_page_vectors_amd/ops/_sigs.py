"""ctypes prototypes of the HIP launcher ABI (csrc/kernels/*.hip).

Codes: p = pointer, i = int32, u = uint32, l = int64, f = float32.
Every launcher returns an int status (0 = ok, >0 hipError_t, <0 argument error).
"""
import ctypes

_T = {"p": ctypes.c_void_p, "i": ctypes.c_int, "u": ctypes.c_uint, "l": ctypes.c_long, "f": ctypes.c_float}

SIGS = {
    # conv_pool_fwd.hip
    "pv_conv_prep_multi": "ippppppip",
    "pv_conv_pack_weights": "ppipp",
    "pv_conv_weight_rows": "ppipp",
    "pv_conv_packed_size": "",
    "pv_conv_set_dbg": "i",
    "pv_conv_set_short": "i",
    "pv_conv_get_dbg": "",
    # chunkpool.hip (chunked long-page encoder, models/chunked.py)
    "pv_chunk_mean_fwd": "pp" "iiii" "pp" "p",
    "pv_chunk_mean_bwd": "pp" "iii" "p" "p",
    # det.hip (deterministic reduction mode, ops/determinism.py)
    "pv_set_deterministic": "i",
    "pv_get_deterministic": "",
    "pv_conv_pool_fwd": "pppppp" "iii" "upu" "ii" "f" "i" "p",
    "pv_conv_pool_fwd2": "ppppppp" "iii" "upu" "ii" "f" "i" "p" "pi",
    "pv_conv_pool_bwd_rec": "ppp" "i" "f" "p",
    # conv_pool_f32.hip (dtype="fp32": reference-precision conv tower)
    "pv_conv_f32_groups": "",
    "pv_conv_f32_set_v2": "i",
    "pv_conv_f32_set_dxw": "i",
    "pv_conv_f32_chunk": "",
    "pv_conv_f32_emax": "",
    "pv_conv_f32_fwd": "ppppppppp" "iiiiiii" "upu" "ii" "f" "pi" "p",
    "pv_conv_f32_mask": "pli" "upu" "ii" "p",
    "pv_conv_f32_bwd_dw": "ppppppp" "iiiii" "upu" "ii" "f" "pi" "p",
    "pv_conv_f32_bwd_dx": "ppppppp" "iiii" "upu" "ii" "f" "pi" "p",
    "pv_conv_f32_dx_lds_max": "",
    "pv_conv_f32_bwd_dx_lds": "pppppppp" "iiiii" "upu" "ii" "f" "pi" "p",
    # conv_pool_bwd.hip
    "pv_conv_pool_bwd_dw": "ppppp" "ppp" "iiii" "upuiif" "p",
    "pv_conv_pool_bwd_dw2": "ppppp" "pppp" "iiii" "upuiif" "p",
    "pv_conv_pool_bwd_emit3": "ppppppp" "iii" "f" "p",
    "pv_conv_bwd_slots_per_sample": "",
    # conv_pool_bwd.hip: dTable reduce
    "pv_conv_pool_bwd_emit3_u16": "pppppp" "iii" "f" "p",
    "pv_conv_pool_bwd_reduce7_u16": "ppppp" "liiii" "upuii" "p",
    "pv_conv_pool_bwd_reduce7": "ppppp" "liiii" "upuii" "p",
    # radix_sort.hip
    "pv_rsort_set_ipt": "i",
    "pv_rsort_temp_bytes": "lii",
    "pv_rsort_pairs": "plpppp" "lii" "p",
    "pv_conv_r7_set_occ": "i",
    # w2v.hip
    "pv_w2v_train": "pppppp" "ll" "iiii" "u" "f" "i" "p",
    # dense.hip
    "pv_gemm_f32": "pll" "pll" "p" "pl" "iiii" "ii" "p",
    "pv_linear_act": "pipippp" "iiiiii" "p",
    "pv_linear_wgrad": "pipip" "iiiii" "p",
    "pv_linear_dgrad": "pipip" "iii" "p",
    "pv_l2norm_fwd": "pppp" "iii" "p",
    "pv_l2norm_bwd": "ppppp" "ii" "p",
    "pv_l2norm_bwd_ld": "pppp" "l" "p" "ii" "p",
    "pv_act_bwd_rowscale": "pppp" "p" "lli" "p",
    "pv_act_bwd2": "ppppl" "ip",
    "pv_act_bwd": "ppp" "li" "p",
    # loss.hip
    "pv_dssm_explicit": "pppppp" "iii" "ffi" "p",
    "pv_ib_fwd": "pppp" "iii" "fi" "ppp" "p",
    "pv_ib_fwd_ws": "iii",
    "pv_ib_bwd": "ppppp" "iii" "fii" "p",
    "pv_ib_bwd_ws": "iii",
    "pv_attn_fwd": "pppp" "iii" "f" "p",
    "pv_attn_bwd": "ppppppp" "iii" "f" "p",
    "pv_attn_bwd2": "ppppppp" "iii" "f" "p" "p",
    "pv_ib_fwd_dq_parts": "ii",
    "pv_ib_fwd_dq": "pppppp" "iiif" "i" "ppp" "p",
    "pv_ib_pos": "ppppppp" "ii" "fi" "p",
    "pv_ib_rows_blk": "p" "iii" "pp" "fi" "p",
    "pv_ib_rowsum": "pp" "ii" "ppp" "f" "p",
    "pv_ib_version": "",
    "pv_ib_fwd_dq2": "ppppppp" "iii" "f" "i" "pppppp" "p",
    "pv_ib_grad_scale_pos": "pifpifpipppppp" "ip",
    "pv_ib_bwd_dd_pos": "ppppp" "iii" "f" "i" "ppp" "p",
    "pv_ib_set_version": "i",
    # embedding.hip
    "pv_trigram_hash": "ppp" "iiii" "p",
    "pv_embedding_bag": "ppppp" "pi" "iiiiii" "p",
    "pv_bag_bwd_sorted": "ppppp" "liiiii" "p",
    "pv_bag_counts": "ppp" "iiiiii" "p",
    # topk.hip
    "pv_topk_splits": "ii",
    "pv_topk_cos": "pppppp" "iiiii" "p",
    # transformer.hip
    "pv_add_layernorm_fwd": "pppppppp" "iif" "p",
    "pv_add_ln_drop_fwd": "ppppppppp" "iif" "ifup" "p",
    "pv_layernorm_bwd_drop": "ppppppp" "pppp" "ii" "ifup" "p",
    "pv_layernorm_bwd_ws": "ii",
    "pv_layernorm_bwd": "ppppppppp" "ii" "p",
    "pv_bias_gelu_fwd": "ppp" "li" "p",
    # lt_gemm.hip (hipBLASLt with fused epilogues)
    "pv_attn_set_qg": "iii",
    "pv_attn_set_fwd_dma": "i",
    "pv_gemm_mx8_set_stages": "i",
    "pv_gelu_set_v": "i",
    "pv_ln_set_rpw": "i",
    "pv_ln_bwd_set_pf": "i",
    "pv_bert_embed_fwd": "ppppp" "li" "ppi" "p",
    "pv_bert_embed_wgrad": "ppp" "li" "p",
    "pv_transpose_u8": "pl" "ii" "pl" "p",
    # loss.hip wide-vector (D = 768) flash passes
    "pv_ibw_splits": "ii",
    "pv_ibw_ws": "iii",
    "pv_ibw": "pi" "pi" "i" "p" "f" "i" "i" "pp" "p",
    "pv_bias_gelu_bwd": "pppppp" "ii" "p",
    "pv_bias_gelu_bwd_ws": "ii",
    "pv_softmax_fwd": "pp" "liif" "p",
    "pv_softmax_bwd": "pp" "lif" "p",
    # fp8.hip
    "pv_amax": "plpp",
    "pv_amax_quant_fp8": "plppp" "pp",
    "pv_quant_fp8": "ppp" "l" "p",
    "pv_fp8_linear": "ppppppp" "iiii" "p",
    # optim.hip
    "pv_adam_dev": "pppp" "l" "p" "fffff" "i" "p" "p",
    "pv_loss_stats": "pp" "i" "pp" "p",
    "pv_ib_grad_scale": "p" "i" "f" "p" "i" "f" "p" "i" "ppp" "p",
    "pv_colsum": "p" "i" "lll" "p" "i" "pp" "ii" "p",
    "pv_adam_set_grid": "i",
    "pv_step_inc": "p" "p",
    "pv_adam_seg": "pppp" "li" "p" "fffff" "i" "pp" "p",
    "pv_adam_rows": "pppp" "i" "pl" "p" "fffff" "i" "pp" "p",
    "pv_adam": "pppp" "li" "fffff" "i" "p" "p",
    "pv_cast_pad_bf16": "pp" "lii" "p",
    "pv_sumsq": "p" "l" "p" "p",
    "pv_scale": "p" "lf" "p",
    # gemm_mx8.hip
    "pv_mx_probe": "ppppp" "p",
    "pv_gemm_mx8": "p" "l" "p" "l" "p" "l" "iii" "i" "l" "p" "f" "p" "ii" "p",
    "pv_amax_quant_fp8_t": "p" "ii" "ppp" "i" "p",
    "pv_bag_counts8": "p" "p" "i" "p" "i" "p" "iiii" "p",
    # bag_gemm.hip (long-bag products with on-the-fly counts)
    "pv_bagd_fwd": "pipp" "iiii" "p",
    "pv_bagd_splits": "iiiii",
    "pv_bagd_wgrad": "pippp" "ii" "iii" "p",
}

_RESTYPE = {"pv_rsort_temp_bytes": ctypes.c_long, "pv_ib_fwd_dq_parts": ctypes.c_long, "pv_ib_bwd_ws": ctypes.c_long, "pv_ib_fwd_ws": ctypes.c_long,
            "pv_bias_gelu_bwd_ws": ctypes.c_long, "pv_layernorm_bwd_ws": ctypes.c_long,
            "pv_ibw_ws": ctypes.c_long}


def declare(lib) -> None:
    for name, codes in SIGS.items():
        fn = getattr(lib, name, None)
        if fn is None:
            continue
        fn.argtypes = [_T[c] for c in codes]
        fn.restype = _RESTYPE.get(name, ctypes.c_int)
