"""Tensor-level wrappers over the libvcg_hip C ABI.

Every wrapper checks device / dtype / contiguity, passes raw device pointers plus sizes, and
launches on torch's current HIP stream. There is no CPU or ATen fallback: a non-GPU tensor or
a missing library raises.
"""
import os

import torch

from . import _lib

F32, BF16 = 0, 1
ACT_NONE, ACT_RELU, ACT_GELU, ACT_TANH, ACT_GELU_BWD = 0, 1, 2, 3, 4
ACT_FLAG_ROUND_PRE = 0x100  # gemm: round alpha*AB + bias to the storage dtype before the residual (vcg_hip.h)
ACT_FLAG_WIDE = 0x200  # gemm: the wide-tile engine (BERT's Linear layers, the downsample dgrad; vcg_hip.h VCG_ACT_FLAG_WIDE)
ACT_FLAG_F32_OUT = 0x400  # gemm (wide, bf16 operands): fp32 residual and output (vcg_hip.h VCG_ACT_FLAG_F32_OUT)
GRAD_F32 = 0x10  # ln_bwd dtype flag: fp32 dout / dres beside bf16 x / res / dx (vcg_hip.h VCG_GRAD_F32)

_DT = {torch.float32: F32, torch.bfloat16: BF16}


def dt_code(dtype):
    try:
        return _DT[dtype]
    except KeyError:
        raise TypeError(f"unsupported storage dtype {dtype}; expected float32 or bfloat16")


def torch_dtype(precision):
    return {"fp32": torch.float32, "bf16": torch.bfloat16}[precision]


def stream():
    return torch.cuda.current_stream().cuda_stream


def P(t):
    """Device pointer of a contiguous GPU tensor (None passes NULL)."""
    if t is None:
        return None
    if not t.is_cuda:
        raise RuntimeError("libvcg_hip ops need GPU tensors (no CPU fallback)")
    return t.data_ptr()


def _chk(t, dtype=None, name="tensor"):
    if not t.is_cuda:
        raise RuntimeError(f"{name} must be on the GPU (libvcg_hip has no CPU path)")
    if not t.is_contiguous():
        raise RuntimeError(f"{name} must be contiguous")
    if dtype is not None and t.dtype != dtype:
        raise RuntimeError(f"{name} has dtype {t.dtype}, expected {dtype}")


def ws(nbytes, device):
    return torch.empty((max(int(nbytes), 4) + 3) // 4, dtype=torch.float32, device=device)


# ----------------------------------------------------------------------------- engine
def conv_out_hw(H, W, KH, KW, stride, pad):
    return (H + 2 * pad - KH) // stride + 1, (W + 2 * pad - KW) // stride + 1


TIMING_FAST_GEMM, TIMING_WGRAD, TIMING_GENERIC_GEMM, TIMING_PATCH_CONV, TIMING_WIDE_GEMM = 0, 1, 2, 3, 4


def gemm_census_enable(on):
    """Start (or stop) counting GEMM-class launches per (kernel, shape); clears the counts."""
    _lib.call("vcg_gemm_census_enable", int(bool(on)))


def gemm_census():
    """{"<kernel tag> M=.. N=.. K=..": launches} since gemm_census_enable(True)."""
    import ctypes
    out = {}
    for i in range(_lib.query("vcg_gemm_census_size")):
        buf = ctypes.create_string_buffer(256)
        n = ctypes.c_longlong()
        _lib.call("vcg_gemm_census_get", i, buf, 256, ctypes.addressof(n))
        out[buf.value.decode()] = n.value
    return out


def timing_enable(on):
    """Bracket every fast-GEMM / wgrad launch with HIP events (clears earlier records)."""
    _lib.call("vcg_timing_enable", int(bool(on)))


def timing_query(kernel_id):
    """(total ms, launches, algorithmic FLOPs) of the recorded launches of one kernel."""
    import ctypes
    ms, n, fl = ctypes.c_double(), ctypes.c_longlong(), ctypes.c_double()
    _lib.call("vcg_timing_query", int(kernel_id), ctypes.addressof(ms), ctypes.addressof(n), ctypes.addressof(fl))
    return ms.value, n.value, fl.value


def timing_roofline(kernel_id, peak_tflops, peak_gbs):
    """(total ms, ideal ms, algorithmic bytes, flops) of the recorded launches of one kernel; ideal = sum of
    max(flops / peak, bytes / HBM peak) per launch."""
    import ctypes
    ms, ideal, nb, fl = ctypes.c_double(), ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
    _lib.call("vcg_timing_roofline", int(kernel_id), float(peak_tflops), float(peak_gbs), ctypes.addressof(ms),
              ctypes.addressof(ideal), ctypes.addressof(nb), ctypes.addressof(fl))
    return ms.value, ideal.value, nb.value, fl.value


def stats_tiles(M):
    return _lib.query("vcg_conv_stats_tiles", M)


def stats_buffer(Cout, M, device):
    """BN statistics buffer of vcg_conv_fwd: float2 [Cout + 1][slots] — (mean, M2) per column and
    slot, then the count row (rows per slot; 0 = unused slot)."""
    return torch.empty((Cout + 1, stats_tiles(M), 2), dtype=torch.float32, device=device)


def conv_fwd(x, w, N, H, W, C, Cout, KH, KW, stride, pad, tsm_T=0, tsm_fold=0, stats=None, out=None):
    """x: NHWC [N,H,W,C]; w: [Cout,KH,KW,C] (same storage dtype). Returns y [N,OH,OW,Cout].
    stats: None or a stats_buffer(Cout, N*OH*OW)."""
    _chk(x, name="x")
    if stats is not None:
        OH_, OW_ = conv_out_hw(H, W, KH, KW, stride, pad)
        if stats.numel() < (Cout + 1) * stats_tiles(N * OH_ * OW_) * 2:
            raise ValueError("stats buffer too small: use ops.stats_buffer(Cout, M)")
    _chk(w, x.dtype, "w")
    OH, OW = conv_out_hw(H, W, KH, KW, stride, pad)
    y = out if out is not None else torch.empty((N, OH, OW, Cout), dtype=x.dtype, device=x.device)
    _lib.call("vcg_conv_fwd", dt_code(x.dtype), P(x), P(w), P(y), P(stats), N, H, W, C, Cout, KH, KW, stride, pad,
              tsm_T, tsm_fold, stream())
    return y


def conv_fwd_bias_act(x, w, bias, act, N, H, W, C, Cout, KH, KW, stride, pad, tsm_T=0, tsm_fold=0, out=None):
    """act(conv(x, w) + bias) (vcg_conv_fwd_bias_act): w carries a folded running-statistics BN, bias its shift."""
    _chk(x, name="x")
    _chk(w, x.dtype, "w")
    _chk(bias, torch.float32, "bias")
    OH, OW = conv_out_hw(H, W, KH, KW, stride, pad)
    y = out if out is not None else torch.empty((N, OH, OW, Cout), dtype=x.dtype, device=x.device)
    _lib.call("vcg_conv_fwd_bias_act", dt_code(x.dtype), P(x), P(w), P(bias), int(act), P(y), N, H, W, C, Cout, KH,
              KW, stride, pad, tsm_T, tsm_fold, stream())
    return y


def conv_dgrad(dy, wt, N, H, W, C, Cout, KH, KW, stride, pad, out=None):
    """dy: NHWC [N,OH,OW,Cout]; wt: [C,KH,KW,Cout]. Returns dx [N,H,W,C]."""
    _chk(dy, name="dy")
    _chk(wt, dy.dtype, "wt")
    dx = out if out is not None else torch.empty((N, H, W, C), dtype=dy.dtype, device=dy.device)
    _lib.call("vcg_conv_dgrad", dt_code(dy.dtype), P(dy), P(wt), P(dx), N, H, W, C, Cout, KH, KW, stride, pad,
              stream())
    return dx


def conv_dgrad_bwd(dy, wt, N, H, W, C, Cout, KH, KW, stride, pad, tsm_T=0, tsm_fold=0, res=None, res_stride=1,
                   bits=None, y=None, mean=None, invstd=None, mscale=None, mshift=None, y2=None, mean2=None, invstd2=None, sums=None,
                   sum_gx2=None, dgamma=None, dbeta=None, dgamma2=None, dbeta2=None, out=None, workspace=None, a2=None,
                   pg=None):
    """Conv input gradient fused with the trunk backward's next steps (vcg_conv_dgrad_bwd, igemm.h BwdEpi):
    g = mask(tsm_adjoint(dgrad) + res) and the BN-backward sums of g against y (sums [2, C] = sum_g,
    sum_gx) and y2 (res_stride 2: res is the compact [N, H/2, W/2, C] gradient of a 1x1 / stride-2 conv) (sum_gx2 [C]); dgamma/dbeta (dgamma2/dbeta2) accumulate. Returns g, or None where the
    fused engine does not apply (fp32 / unsupported shape): the caller then runs the unfused ops.
    a2 (bf16 [N, H, W, a2_c], a2_c 64) with pg (f32 [C, a2_c]): also pg = g^T a2 from the stored g tiles; then
    the return value is (g, done) -- done False where that product does not apply (g computed without it)."""
    OH, OW = conv_out_hw(H, W, KH, KW, stride, pad)
    _chk(dy, None, "dy")
    assert dy.numel() == N * OH * OW * Cout and wt.numel() == C * KH * KW * Cout
    g = out if out is not None else torch.empty((N, H, W, C), dtype=dy.dtype, device=dy.device)
    nbytes = _lib.query("vcg_conv_dgrad_bwd_ws_bytes", C, Cout, KH, KW)
    if workspace is None or workspace.numel() * 4 < nbytes:
        workspace = ws(nbytes, dy.device)
    for t in (res, y, y2):
        if t is not None:
            _chk(t, dy.dtype)
            assert t.numel() == (N * ((H + 1) // 2) * ((W + 1) // 2) * C if t is res and res_stride == 2
                                 else N * H * W * C)
    def call(a2_, pg_, pws_):
        return _lib.query("vcg_conv_dgrad_bwd", dt_code(dy.dtype), P(dy), P(wt), P(g), N, H, W, C, Cout, KH, KW,
                          stride, pad, tsm_T, tsm_fold, P(res), int(res_stride), P(bits), P(y), P(mean), P(invstd),
                          P(mscale), P(mshift), P(y2), P(mean2), P(invstd2), P(workspace), workspace.numel() * 4,
                          P(sums[0]) if sums is not None else None, P(sums[1]) if sums is not None else None,
                          P(dgamma), P(dbeta), P(sum_gx2), P(dgamma2), P(dbeta2), P(a2_),
                          a2_.shape[-1] if a2_ is not None else 0, P(pg_), P(pws_),
                          pws_.numel() * 4 if pws_ is not None else 0, stream())
    done = False
    rc = -2
    if a2 is not None:
        _chk(a2, torch.bfloat16, "a2")
        _chk(pg, torch.float32, "pg")
        assert a2.numel() == N * H * W * a2.shape[-1] and pg.numel() == C * a2.shape[-1]
        pws = ws(_lib.query("vcg_conv_dgrad_bwd_p_ws_bytes", C, a2.shape[-1]), dy.device)
        rc = call(a2, pg, pws)
        done = rc == 0
    if rc == -2:  # VCG_ERR_UNSUPPORTED (with a2: retried without the P product)
        rc = call(None, None, None)
    if rc == -2:
        return (None, False) if a2 is not None else None
    if rc != 0:
        raise _lib.VcgError(f"vcg_conv_dgrad_bwd failed ({rc}): {_lib.last_error()}")
    return (g, done) if a2 is not None else g


def bn_apply_colsum(y, scale, shift, C, relu=True):
    """(bn_apply(y, scale, shift, relu), its column sums f32 [C]) in one pass (vcg_bn_apply_colsum, bf16)."""
    _chk(y, torch.bfloat16, "y")
    out = torch.empty_like(y)
    cs = torch.empty(C, dtype=torch.float32, device=y.device)
    P_ = y.numel() // C
    w = ws(_lib.query("vcg_bn_apply_colsum_ws_bytes", P_, C), y.device)
    _lib.call("vcg_bn_apply_colsum", P(y), P(scale), P(shift), int(relu), P(out), P(cs), P(w), w.numel() * 4, P_, C,
              stream())
    return out, cs


def bn_apply_gram(y, scale, shift, C, mean, invstd):
    """(relu(bn_apply(y)), its column sums f32 [C], its Gram matrix out^T out f32 [C, C], and g64: the same Gram
    matrix and column sums accumulated centred per channel, with the centres, double [C * C + 2 C]) in one pass
    (vcg_bn_apply_gram, bf16, C in 64 / 128 / 256; mean / invstd: the BN statistics scale / shift fold; g64 is what
    bn_stats_from_gram reads)."""
    _chk(y, torch.bfloat16, "y")
    out = torch.empty_like(y)
    cs = torch.empty(C, dtype=torch.float32, device=y.device)
    gram = torch.empty((C, C), dtype=torch.float32, device=y.device)
    g64 = torch.empty(C * C + 2 * C, dtype=torch.float64, device=y.device)
    P_ = y.numel() // C
    w = ws(_lib.query("vcg_bn_apply_gram_ws_bytes", P_, C), y.device)
    _lib.call("vcg_bn_apply_gram", P(y), P(scale), P(shift), P(mean), P(invstd), P(out), P(cs), P(gram), P(g64),
              P(w), w.numel() * 4, P_, C, stream())
    return out, cs, gram, g64


def bn_stats_from_gram(g64, w, M, N, C, stats):
    """BN statistics of x w^T (w bf16 [N, C]) from x's centred (Gram matrix, column sums, centres) g64 [C * C + 2 C]
    of bn_apply_gram into a stats_buffer(N, M) (vcg_bn_stats_from_gram; one used slot, for bn_finalize)."""
    _chk(w, torch.bfloat16, "w")
    _chk(g64, torch.float64, "g64")
    assert g64.numel() == C * C + 2 * C
    _lib.call("vcg_bn_stats_from_gram", P(g64), P(w), M, N, C, P(stats), stats.shape[1], stream())
    return stats


def bn_finalize_from_gram(g64, w, M, N, C, gamma, beta, mean, invstd, scale, shift, running_mean=None,
                          running_var=None, momentum=0.1, eps=1e-5, w32=None, wfold=None):
    """bn_stats_from_gram + bn_finalize (+ weight_fold of the f32 master weight w32 [N, C] by the new scale into wfold,
    bf16) in one launch (vcg_bn_finalize_from_gram; the same values as the three calls). C <= 256, C % 16 == 0."""
    _chk(w, torch.bfloat16, "w")
    _chk(g64, torch.float64, "g64")
    assert g64.numel() == C * C + 2 * C and C <= 256 and C % 16 == 0
    if w32 is not None:
        _chk(w32, torch.float32, "w32")
        _chk(wfold, torch.bfloat16, "wfold")
        assert w32.numel() == N * C and wfold.numel() == N * C
    _lib.call("vcg_bn_finalize_from_gram", P(g64), P(w), M, N, C, P(gamma), P(beta), P(mean), P(invstd), P(scale),
              P(shift), P(running_mean), P(running_var), float(momentum), float(eps), P(w32), P(wfold), stream())


def conv1x1_stats(x, w, stats, M, N, K):
    """BatchNorm statistics of x [M, K] @ w [N, K]^T without storing the product (vcg_conv1x1_stats). False where
    the fused engine does not apply."""
    _chk(x, torch.bfloat16, "x")
    _chk(w, torch.bfloat16, "w")
    rc = _lib.query("vcg_conv1x1_stats", P(x), P(w), P(stats), M, N, K, stream())
    if rc == -2:
        return False
    if rc != 0:
        raise _lib.VcgError(f"vcg_conv1x1_stats failed ({rc}): {_lib.last_error()}")
    return True


def bn_bwd_sumgx_from_wgrad(Pg, w, K, C, mean, invstd, sum_g, sum_gx, dgamma=None):
    """sum_gx of a BN whose input y3 = a2 w^T was not stored, from Pg = g^T a2 (vcg_bn_bwd_sumgx_from_wgrad)."""
    _chk(Pg, torch.float32, "Pg")
    _chk(w, torch.bfloat16, "w")
    _lib.call("vcg_bn_bwd_sumgx_from_wgrad", P(Pg), P(w), K, C, P(mean), P(invstd), P(sum_g), P(sum_gx), P(dgamma),
              stream())


def conv1x1_bn_res_relu(x, wfold, bias, res, M, N, K, res_scale=None, res_shift=None):
    """(out, bits): relu(bf16(x @ wfold^T + bias) + res') and its ReLU mask bits (vcg_conv1x1_bn_res_relu), res' =
    res or res * res_scale + res_shift per column; None where the fused engine does not apply."""
    _chk(x, torch.bfloat16, "x")
    _chk(res, torch.bfloat16, "res")
    out = torch.empty_like(res)
    bits = torch.empty(res.numel() // 8, dtype=torch.uint8, device=res.device)
    rc = _lib.query("vcg_conv1x1_bn_res_relu", P(x), P(wfold), P(bias), P(res), P(res_scale), P(res_shift), P(out),
                    P(bits), M, N, K, stream())
    if rc == -2:
        return None
    if rc != 0:
        raise _lib.VcgError(f"vcg_conv1x1_bn_res_relu failed ({rc}): {_lib.last_error()}")
    return out, bits


def bn_bwd_fold_weights(wt, N, K, mean, invstd, gamma, sum_g, sum_gx, count):
    """(wfold [N, 2K] bf16, bias [N] f32) of a batch-statistics BN backward folded into the dgrad whose B operand is
    wt [N, K] (vcg_bn_bwd_fold_weights)."""
    _chk(wt, torch.bfloat16, "wt")
    wfold = torch.empty((N, 2 * K), dtype=torch.bfloat16, device=wt.device)
    bias = torch.empty(N, dtype=torch.float32, device=wt.device)
    _lib.call("vcg_bn_bwd_fold_weights", P(wt), N, K, P(mean), P(invstd), P(gamma), P(sum_g), P(sum_gx),
              float(1.0 / count), P(wfold), P(bias), stream())
    return wfold, bias


def conv_dgrad_bwd_bnfold(g, yg, wfold, bias, N, H, W, C, Cout, y=None, mean=None, invstd=None, mscale=None,
                          mshift=None, sums=None, dgamma=None, dbeta=None, out=None, workspace=None, Ky=None):
    """Input gradient of a 1x1 conv whose output gradient is the folded BN backward (vcg_conv_dgrad_bwd_bnfold; the
    light epilogue of conv_dgrad_bwd): one GEMM over [g | yg], yg = the BN input y (Ky = Cout, bn_bwd_fold_weights) or
    the conv's input a2 (Ky = C, bn_bwd_fold_weights_a2). Returns the masked gradient, or None where the engine does
    not apply."""
    Ky = Cout if Ky is None else Ky
    _chk(g, torch.bfloat16, "g")
    _chk(yg, torch.bfloat16, "yg")
    assert g.numel() == N * H * W * Cout and yg.numel() == N * H * W * Ky and wfold.numel() == C * (Cout + Ky)
    gout = out if out is not None else torch.empty((N, H, W, C), dtype=g.dtype, device=g.device)
    nbytes = _lib.query("vcg_conv_dgrad_bwd_ws_bytes", C, Cout + Ky, 1, 1)
    if workspace is None or workspace.numel() * 4 < nbytes:
        workspace = ws(nbytes, g.device)
    rc = _lib.query("vcg_conv_dgrad_bwd_bnfold", P(g), P(yg), int(Ky), P(wfold), P(bias), P(gout), N, H, W, C, Cout, P(y),
                    P(mean), P(invstd), P(mscale), P(mshift), P(workspace), workspace.numel() * 4,
                    P(sums[0]) if sums is not None else None, P(sums[1]) if sums is not None else None, P(dgamma),
                    P(dbeta), stream())
    if rc == -2:
        return None
    if rc != 0:
        raise _lib.VcgError(f"vcg_conv_dgrad_bwd_bnfold failed ({rc}): {_lib.last_error()}")
    return gout


def bn_bwd_fold_weights_a2(wt, C, K, invstd, gamma, sum_g, sum_gx, count, colsum_a):
    """(wfold [C, K + C] bf16, bias [C] f32) of the BN backward folded into the dgrad with the conv input a2 as the
    second source (vcg_bn_bwd_fold_weights_a2)."""
    _chk(wt, torch.bfloat16, "wt")
    wfold = torch.empty((C, K + C), dtype=torch.bfloat16, device=wt.device)
    bias = torch.empty(C, dtype=torch.float32, device=wt.device)
    _lib.call("vcg_bn_bwd_fold_weights_a2", P(wt), C, K, P(invstd), P(gamma), P(sum_g), P(sum_gx), float(1.0 / count),
              P(colsum_a), P(wfold), P(bias), stream())
    return wfold, bias


def bn_bwd_fold_wgrad_a2(Pg, G, w3, K, C, mean, invstd, gamma, sum_g, sum_gx, count, colsum_a, dw, accumulate=True):
    """dw [K, C] (+)= A Pg + B (w3 G) + Cc colsum_a (vcg_bn_bwd_fold_wgrad_a2)."""
    for t, n in ((Pg, "Pg"), (G, "G"), (w3, "w3"), (dw, "dw")):
        _chk(t, torch.float32, n)
    _lib.call("vcg_bn_bwd_fold_wgrad_a2", P(Pg), P(G), P(w3), K, C, P(mean), P(invstd), P(gamma), P(sum_g), P(sum_gx),
              float(1.0 / count), P(colsum_a), P(dw), int(accumulate), stream())


def conv_wgrad_bnfold(x, g, yg, mean, invstd, gamma, sum_g, sum_gx, count, colsum_x, dw, N, H, W, C, Cout,
                      accumulate=True, workspace=None):
    """dw [Cout, C] (+)= weight gradient of a 1x1 conv over x whose output gradient is the folded BN backward
    (vcg_conv_wgrad_bnfold). Returns False where the engine does not apply."""
    _chk(x, torch.bfloat16, "x")
    _chk(dw, torch.float32, "dw")
    nbytes = _lib.query("vcg_conv_wgrad_bnfold_ws_bytes", N, H, W, C, Cout)
    if workspace is None or workspace.numel() * 4 < nbytes:
        workspace = ws(nbytes, x.device)
    rc = _lib.query("vcg_conv_wgrad_bnfold", P(x), P(g), P(yg), P(mean), P(invstd), P(gamma), P(sum_g), P(sum_gx),
                    float(1.0 / count), P(colsum_x), P(dw), int(accumulate), P(workspace), workspace.numel() * 4, N, H,
                    W, C, Cout, stream())
    if rc == -2:
        return False
    if rc != 0:
        raise _lib.VcgError(f"vcg_conv_wgrad_bnfold failed ({rc}): {_lib.last_error()}")
    return True


def conv_wgrad(x, dy, dw, N, H, W, C, Cin, Cout, KH, KW, stride, pad, tsm_T=0, tsm_fold=0, accumulate=True,
               workspace=None):
    """dw (fp32 OIHW [Cout,Cin,KH,KW]) += wgrad. x: NHWC with C (padded) channels."""
    _chk(x, name="x")
    _chk(dy, x.dtype, "dy")
    _chk(dw, torch.float32, "dw")
    nbytes = _lib.query("vcg_conv_wgrad_ws_bytes", dt_code(x.dtype), N, H, W, C, Cout, KH, KW, stride, pad)
    if workspace is None or workspace.numel() * 4 < nbytes:
        workspace = ws(nbytes, x.device)
    _lib.call("vcg_conv_wgrad", dt_code(x.dtype), P(x), P(dy), P(dw), int(accumulate), P(workspace),
              workspace.numel() * 4, N, H, W, C, Cin, Cout, KH, KW, stride, pad, tsm_T, tsm_fold, stream())
    return workspace


def conv_wgrad_ws_bytes(dtype, N, H, W, C, Cout, KH, KW, stride, pad):
    return _lib.query("vcg_conv_wgrad_ws_bytes", dt_code(dtype), N, H, W, C, Cout, KH, KW, stride, pad)


def gemm(A, B, M, N, K, lda, ldb, transA=False, transB=False, out=None, ldc=None, bias=None, act=ACT_NONE,
         residual=None, ldr=None, aux=None, alpha=1.0):
    """C[M,N] = act(alpha * op(A) @ op(B)^T + bias (+ residual)). A/B/C share the storage dtype.
    transA=False: A is [M][lda]; True: A is [K][lda]. transB=False: B is [N][ldb]; True: [K][ldb]."""
    if out is None:
        out = torch.empty((M, N), dtype=A.dtype, device=A.device)
        ldc = N
    ldc = ldc if ldc is not None else N
    _lib.call("vcg_gemm", dt_code(A.dtype), int(transA), int(transB), M, N, K, P(A), lda, P(B), ldb, P(out), ldc,
              P(bias), act, P(residual), ldr if ldr is not None else ldc, P(aux), float(alpha), stream())
    return out


def gemm_batched(A, B, C, M, N, K, lda, ldb, ldc, a_so, a_si, b_so, b_si, c_so, c_si, batch_outer, batch_inner,
                 transA=False, transB=False, bias=None, act=ACT_NONE, alpha=1.0):
    _lib.call("vcg_gemm_batched", dt_code(A.dtype), int(transA), int(transB), M, N, K, P(A), lda, a_so, a_si, P(B),
              ldb, b_so, b_si, P(C), ldc, c_so, c_si, batch_outer, batch_inner, P(bias), act, float(alpha), stream())
    return C


def gemm_splitk(A, B, out, M, N, K, lda, ldb, transA=False, transB=False, accumulate=True, workspace=None):
    """out (fp32 [M,N]) (+)= op(A) @ op(B)^T, split over K."""
    _chk(out, torch.float32, "out")
    nbytes = _lib.query("vcg_gemm_splitk_ws_bytes", dt_code(A.dtype), M, N, K)
    if workspace is None or workspace.numel() * 4 < nbytes:
        workspace = ws(nbytes, A.device)
    _lib.call("vcg_gemm_splitk", dt_code(A.dtype), int(transA), int(transB), M, N, K, P(A), lda, P(B), ldb, P(out),
              int(accumulate), P(workspace), workspace.numel() * 4, stream())
    return workspace


# ----------------------------------------------------------------------------- vision
def bn_finalize(stats, mtiles, M, C, gamma, beta, mean, invstd, scale, shift, running_mean=None, running_var=None,
                momentum=0.1, eps=1e-5):
    _lib.call("vcg_bn_finalize", P(stats), mtiles, M, C, P(gamma), P(beta), P(mean), P(invstd), P(scale), P(shift),
              P(running_mean), P(running_var), float(momentum), float(eps), stream())


def bn_eval_params(gamma, beta, rm, rv, eps, C, mean, invstd, scale, shift):
    _lib.call("vcg_bn_eval_params", P(gamma), P(beta), P(rm), P(rv), float(eps), C, P(mean), P(invstd), P(scale),
              P(shift), stream())


def bn_apply(y, scale, shift, C, relu, res=None, rscale=None, rshift=None, out=None, bits=False):
    """act(y*scale + shift [+ res*rscale + rshift | + res]). bits=True also returns the ReLU mask
    bits of the output (one byte per 16-B vector) for the backward (mask mode 2)."""
    out = out if out is not None else torch.empty_like(y)
    b = torch.empty(y.numel() * y.element_size() // 16, dtype=torch.uint8, device=y.device) if bits else None
    _lib.call("vcg_bn_apply", dt_code(y.dtype), P(y), P(scale), P(shift), P(res), P(rscale), P(rshift), int(relu),
              P(out), P(b), y.numel() // C, C, stream())
    return (out, b) if bits else out


def _mask_mode(mask, mbits, mscale):
    if mbits is not None:
        return 2
    if mscale is not None:
        return 3
    return 1 if mask is not None else 0


def bn_bwd_reduce(dout, mask, y, mean, invstd, C, sum_g, sum_gx, dgamma=None, dbeta=None, workspace=None,
                  mbits=None, mscale=None, mshift=None):
    """Per-channel sums of g and g*xhat, g = dout masked by the ReLU: `mask` tensor (> 0), `mbits`
    (from bn_apply(bits=True)) or the affine recompute fma(y, mscale, mshift) > 0."""
    Pn = y.numel() // C
    nbytes = _lib.query("vcg_bn_bwd_ws_bytes", Pn, C)
    if workspace is None or workspace.numel() * 4 < nbytes:
        workspace = ws(nbytes, y.device)
    _lib.call("vcg_bn_bwd_reduce", dt_code(y.dtype), P(dout), _mask_mode(mask, mbits, mscale), P(mask), P(mbits),
              P(mscale), P(mshift), P(y), P(mean), P(invstd), Pn, C, P(workspace), workspace.numel() * 4, P(sum_g),
              P(sum_gx), P(dgamma), P(dbeta), 1, stream())
    return workspace


def bn_bwd_apply(dout, mask, y, mean, invstd, gamma, sum_g, sum_gx, C, train_stats, gout=None, out=None,
                 mbits=None, mscale=None, mshift=None):
    Pn = y.numel() // C
    dy = out if out is not None else torch.empty_like(y)
    _lib.call("vcg_bn_bwd_apply", dt_code(y.dtype), P(dout), _mask_mode(mask, mbits, mscale), P(mask), P(mbits),
              P(mscale), P(mshift), P(y), P(mean), P(invstd), P(gamma), P(sum_g), P(sum_gx), Pn, int(train_stats),
              P(dy), P(gout), Pn, C, stream())
    return dy


def bn_bwd_apply_dual(g, y, mean, invstd, gamma, sum_g, sum_gx, yd, mean_d, invstd_d, gamma_d, sum_g_d, sum_gx_d,
                      C):
    """Batch-stat BN backward applies of two BNs on one (masked) gradient g: (dy, dyd), g read once."""
    Pn = y.numel() // C
    dy, dyd = torch.empty_like(y), torch.empty_like(yd)
    _lib.call("vcg_bn_bwd_apply_dual", dt_code(y.dtype), P(g), P(y), P(mean), P(invstd), P(gamma), P(sum_g),
              P(sum_gx), P(yd), P(mean_d), P(invstd_d), P(gamma_d), P(sum_g_d), P(sum_gx_d), Pn, P(dy), P(dyd), Pn, C,
              stream())
    return dy, dyd


def maxpool_fwd(x, N, H, W, C):
    OH, OW = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    y = torch.empty((N, OH, OW, C), dtype=x.dtype, device=x.device)
    idx = torch.empty((N, OH, OW, C), dtype=torch.uint8, device=x.device)
    _lib.call("vcg_maxpool_fwd", dt_code(x.dtype), P(x), P(y), P(idx), N, H, W, C, stream())
    return y, idx


def maxpool_bwd(dy, idx, N, H, W, C):
    dx = torch.empty((N, H, W, C), dtype=dy.dtype, device=dy.device)
    _lib.call("vcg_maxpool_bwd", dt_code(dy.dtype), P(dy), P(idx), P(dx), N, H, W, C, stream())
    return dx


def maxpool_bwd_bn(dy, idx, N, H, W, C, y, mean, invstd, mscale, mshift, sums, dgamma=None, dbeta=None,
                   store_g=True):
    """maxpool backward + the stem BN + ReLU mask + BN-backward sums (sums [2, C] = sum_g, sum_gx). Returns the
    masked gradient g, or None with store_g=False (sums only: maxpool_bwd_bn_apply recomputes g)."""
    g = torch.empty((N, H, W, C), dtype=dy.dtype, device=dy.device) if store_g else None
    w = ws(_lib.query("vcg_maxpool_bwd_bn_ws_bytes", C), dy.device)
    _lib.call("vcg_maxpool_bwd_bn", dt_code(dy.dtype), P(dy), P(idx), P(g), N, H, W, C, P(y), P(mean), P(invstd),
              P(mscale), P(mshift), P(w), w.numel() * 4, P(sums[0]), P(sums[1]), P(dgamma), P(dbeta), stream())
    return g


def maxpool_bwd_bn_sums_pooled(dy, mp, idx, y, N, H, W, C, mean, invstd, mscale, mshift, sums, dgamma=None,
                               dbeta=None):
    """The stem BN-backward sums of maxpool_bwd_bn(store_g=False) from the pooled activation mp (no pass over the
    pre-pool y [N, H, W, C], which -- with the argmax bytes idx -- is read only for channels with a zero or tiny BN
    weight; vcg_maxpool_bwd_bn_sums_pooled)."""
    OH, OW = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    assert tuple(mp.shape) == (N, OH, OW, C) and idx.shape == mp.shape and tuple(y.shape) == (N, H, W, C)
    w = ws(_lib.query("vcg_maxpool_bwd_bn_ws_bytes", C), dy.device)
    _lib.call("vcg_maxpool_bwd_bn_sums_pooled", dt_code(dy.dtype), P(dy), P(mp), P(idx), P(y), N, H, W, C, P(mean),
              P(invstd), P(mscale), P(mshift), P(w), w.numel() * 4, P(sums[0]), P(sums[1]), P(dgamma), P(dbeta),
              stream())


def maxpool_bwd_bn_apply(dy, idx, N, H, W, C, y, mean, invstd, mscale, mshift, gamma, sums, count, train_stats):
    """The stem's BN-backward apply on g = mask(maxpool_bwd(dy)) recomputed in the same pass (sums from
    maxpool_bwd_bn(store_g=False)): returns the gradient of the stem conv output y."""
    dx = torch.empty((N, H, W, C), dtype=dy.dtype, device=dy.device)
    _lib.call("vcg_maxpool_bwd_bn_apply", dt_code(dy.dtype), P(dy), P(idx), P(dx), N, H, W, C, P(y), P(mean),
              P(invstd), P(mscale), P(mshift), P(gamma), P(sums[0]), P(sums[1]), int(count), int(bool(train_stats)),
              stream())
    return dx


def stem_bwd_fused(dy, idx, y, x, N, H, W, mean, invstd, mscale, mshift, gamma, sums, count, train_stats, dw,
                   accumulate=True):
    """The stem backward after the max-pool in one pass (bf16): maxpool_bwd_bn_apply's dy0 contracted with the
    pair-packed frames x [N][2H][2W][4] into dw [64][3][7][7] (vcg_stem_bwd_fused; dy0 is never stored)."""
    for t, n in ((dy, "dy"), (y, "y"), (x, "x")):
        _chk(t, torch.bfloat16, n)
    _chk(dw, torch.float32, "dw")
    assert tuple(y.shape) == (N, H, W, 64) and tuple(x.shape) == (N, 2 * H, 2 * W, 4) and dw.numel() == 64 * 147
    assert tuple(dy.shape) == (N, (H - 1) // 2 + 1, (W - 1) // 2 + 1, 64) and idx.shape == dy.shape
    w = ws(_lib.query("vcg_stem_bwd_fused_ws_bytes"), dy.device)
    _lib.call("vcg_stem_bwd_fused", P(dy), P(idx), P(y), P(x), N, H, W, P(mean), P(invstd), P(mscale), P(mshift),
              P(gamma), P(sums[0]), P(sums[1]), int(count), int(bool(train_stats)), P(w), w.numel() * 4, P(dw),
              int(bool(accumulate)), stream())


def stem_bwd_fused_fits(N, H, W):
    """stem_bwd_fused takes a [N][H][W][64] conv output: every operand below 4 GB (32-bit buffer offsets; host-side
    predicate of the library, vcg_stem_bwd_fused_fits)."""
    return bool(_lib.query("vcg_stem_bwd_fused_fits", int(N), int(H), int(W)))


def bn_relu_maxpool(y, scale, shift, N, H, W, C):
    """maxpool3x3/2(relu(y * scale + shift)) with the activation rounded to y's dtype (the values and argmax of
    bn_apply + maxpool_fwd, without the activation tensor). Returns (pooled, idx)."""
    OH, OW = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    out = torch.empty((N, OH, OW, C), dtype=y.dtype, device=y.device)
    idx = torch.empty((N, OH, OW, C), dtype=torch.uint8, device=y.device)
    _lib.call("vcg_bn_relu_maxpool", dt_code(y.dtype), P(y), P(scale), P(shift), P(out), P(idx), N, H, W, C, stream())
    return out, idx


def avgpool_fwd(x, N, HW, C):
    y = torch.empty((N, C), dtype=torch.float32, device=x.device)
    _lib.call("vcg_avgpool_fwd", dt_code(x.dtype), P(x), P(y), N, HW, C, stream())
    return y


def avgpool_bwd(dy, N, HW, C, dtype):
    dx = torch.empty((N, HW, C), dtype=dtype, device=dy.device)
    _lib.call("vcg_avgpool_bwd", dt_code(dtype), P(dy), P(dx), N, HW, C, stream())
    return dx


IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def stem_cpad(dtype):
    """Channels of the stem's NHWC input: 4 (RGB0; bf16: the pair-packed stem, two stride-2 taps per 16-B chunk,
    vcg_conv_fwd)."""
    return 4


def window_frames_u8(frames, idx, dtype, mean=IMAGENET_MEAN, std=IMAGENET_STD, cpad=8):
    """u8 RGB frames [F,H,W,3] gathered by an int64 frame table `idx` (any shape, 0-based) ->
    normalised NHWC stem input [idx.numel(),H,W,cpad] (channels 3.. zero; cpad 4 or 8)."""
    import ctypes

    _chk(frames, torch.uint8, "frames")
    _chk(idx, torch.int64, "idx")
    F, H, W, C = frames.shape
    if C != 3:
        raise ValueError("frames must be [F,H,W,3] RGB")
    n = idx.numel()
    dst = torch.empty((n, H, W, cpad), dtype=dtype, device=frames.device)
    m = (ctypes.c_float * 3)(*mean)
    sd = (ctypes.c_float * 3)(*std)
    _lib.call("vcg_window_frames_u8_cpad", dt_code(dtype), P(frames), P(idx), P(dst), n, F, H, W, cpad,
              ctypes.addressof(m), ctypes.addressof(sd), stream())
    return dst


def frames_to_nhwc(src, N, C, H, W, Cpad, dtype):
    _chk(src, torch.float32, "frames")
    dst = torch.empty((N, H, W, Cpad), dtype=dtype, device=src.device)
    _lib.call("vcg_frames_to_nhwc", dt_code(dtype), P(src), P(dst), N, C, H, W, Cpad, stream())
    return dst


def pair_taps(KW, pad):
    """(KWp, pwp) of the pair-packed stem (igemm.hip pair_taps): super-pixel taps and pad."""
    lo = (-pad) // 2
    return (KW - 1 - pad) // 2 - lo + 1, -lo


def weight_prep(w, Cpad, dtype, transposed=False, out=None, pair_pad=None):
    """GEMM operand of a conv weight; pair_pad (bf16, Cpad = 4): the pair-packed stem layout for that pad."""
    _chk(w, torch.float32, "weight")
    Cout, Cin, KH, KW = w.shape
    mode = int(transposed)
    if pair_pad is not None:
        shape, mode = (Cout, KH, pair_taps(KW, pair_pad)[0], 8), 2 + pair_pad
    else:
        shape = (Cin, KH, KW, Cout) if transposed else (Cout, KH, KW, Cpad)
    out = out if out is not None else torch.empty(shape, dtype=dtype, device=w.device)
    _lib.call("vcg_weight_prep", dt_code(dtype), P(w), P(out), Cout, Cin, KH, KW, Cpad, mode, stream())
    return out


def weight_fold(w2d, scale, dtype, out=None):
    """[rows, cols] f32 weight with row r scaled by scale[r], cast to dtype (vcg_weight_fold): a running-statistics BN
    folded into the 1x1 conv before it."""
    _chk(w2d, torch.float32, "weight")
    rows, cols = w2d.shape
    out = out if out is not None else torch.empty((rows, cols), dtype=dtype, device=w2d.device)
    _lib.call("vcg_weight_fold", dt_code(dtype), P(w2d), P(scale), P(out), rows, cols, stream())
    return out


def weight_prep_multi(desc, n):
    """One launch of vcg_weight_prep_multi over a DEVICE int64 descriptor table [n, 8]."""
    _chk(desc, torch.int64, "desc")
    assert desc.numel() >= 8 * n
    _lib.call("vcg_weight_prep_multi", BF16, P(desc), int(n), stream())


def transpose_multi(desc, n, total_tiles):
    """One launch of vcg_transpose_multi over a DEVICE int64 descriptor table [n, 5] (src, dst, rows, cols, first
    tile): bf16 [rows][cols] -> [cols][rows]."""
    _chk(desc, torch.int64, "desc")
    assert desc.numel() >= 5 * n
    _lib.call("vcg_transpose_multi", P(desc), int(n), int(total_tiles), stream())


def transpose(x, out=None):
    """[rows, cols] -> [cols, rows] (contiguous)."""
    _chk(x, None, "x")
    rows, cols = x.shape
    out = out if out is not None else torch.empty((cols, rows), dtype=x.dtype, device=x.device)
    _lib.call("vcg_transpose", dt_code(x.dtype), P(x), P(out), rows, cols, cols, rows, stream())
    return out


def cast_from_f32(x, dtype, out=None):
    _chk(x, torch.float32, "x")
    out = out if out is not None else torch.empty(x.shape, dtype=dtype, device=x.device)
    _lib.call("vcg_cast_from_f32", dt_code(dtype), P(x), P(out), x.numel(), stream())
    return out


def cast_to_f32(x, out=None):
    out = out if out is not None else torch.empty(x.shape, dtype=torch.float32, device=x.device)
    _lib.call("vcg_cast_to_f32", dt_code(x.dtype), P(x), P(out), x.numel(), stream())
    return out


def tsm_shift(x, n_segment, fold_div, direction=0):
    """Reference TemporalShift.shift on an NCHW tensor [n_batch*T, C, H, W] (direction 1 = adjoint)."""
    _chk(x, name="x")
    nt, c, h, w = x.shape
    y = torch.empty_like(x)
    _lib.call("vcg_tsm_shift", dt_code(x.dtype), P(x), P(y), nt // n_segment, n_segment, c, h * w, fold_div,
              direction, stream())
    return y


def tsm_unshift_add(dshift, other, NT, T, HW, C, fold, other_bits=None):
    """dx = unshift(dshift) + other (other masked by `other_bits` when given)."""
    dx = torch.empty_like(dshift)
    _lib.call("vcg_tsm_unshift_add", dt_code(dshift.dtype), P(dshift), P(other), P(other_bits), P(dx), NT, T, HW, C,
              fold, stream())
    return dx


# ----------------------------------------------------------------------------- text
def embed_ln_fwd(ids, word, pos, typ, gamma, beta, B, L, H, eps, dtype, p=0.0, seed=0):
    out = torch.empty((B * L, H), dtype=dtype, device=ids.device)
    mean = torch.empty(B * L, dtype=torch.float32, device=ids.device)
    rstd = torch.empty(B * L, dtype=torch.float32, device=ids.device)
    _lib.call("vcg_embed_ln_fwd", dt_code(dtype), P(ids), P(word), P(pos), P(typ), P(gamma), P(beta), P(out), P(mean),
              P(rstd), B, L, H, float(eps), float(p), int(seed) & (2**64 - 1), stream())
    return out, mean, rstd


def embed_ln_bwd(dout, ids, word, pos, typ, gamma, mean, rstd, word_grad, pos_grad, type_grad, gamma_grad, beta_grad,
                 B, L, H, p=0.0, seed=0, pad_idx=-1):
    nbytes = _lib.query("vcg_ln_bwd_ws_bytes", B * L, H)
    w = ws(nbytes, dout.device)
    _lib.call("vcg_embed_ln_bwd", dt_code(dout.dtype), P(dout), P(ids), P(word), P(pos), P(typ), P(gamma), P(mean),
              P(rstd), P(word_grad), P(pos_grad), P(type_grad), P(gamma_grad), P(beta_grad), P(w), w.numel() * 4, B, L,
              H, float(p), int(seed) & (2**64 - 1), int(pad_idx), stream())


def ln_fwd(x, res, gamma, beta, rows, H, eps, p=0.0, seed=0):
    out = torch.empty_like(x)
    mean = torch.empty(rows, dtype=torch.float32, device=x.device)
    rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
    _lib.call("vcg_ln_fwd", dt_code(x.dtype), P(x), P(res), P(gamma), P(beta), P(out), P(mean), P(rstd), rows, H,
              float(eps), float(p), int(seed) & (2**64 - 1), stream())
    return out, mean, rstd


def ln_bwd(dout, x, res, gamma, mean, rstd, gamma_grad, beta_grad, rows, H, p=0.0, seed=0, want_dx=True,
           want_dres=True, bias_grad=None):
    """LayerNorm(dropout(x) + res) backward. bias_grad (optional, accumulated): column sums of dx, i.e. the
    bias gradient of the dense layer that produced x. dx has x's dtype, dres dout's: a bf16 x with an fp32 dout keeps
    the residual gradient in fp32 (VCG_GRAD_F32)."""
    dx = torch.empty_like(x) if want_dx else None
    dres = torch.empty_like(dout) if want_dres else None
    nbytes = _lib.query("vcg_ln_bwd_ws_bytes", rows, H)
    w = ws(nbytes, dout.device)
    code = dt_code(x.dtype)
    if dout.dtype != x.dtype:
        if not (x.dtype == torch.bfloat16 and dout.dtype == torch.float32):
            raise TypeError(f"ln_bwd: dout {dout.dtype} with x {x.dtype}")
        code |= GRAD_F32
    _lib.call("vcg_ln_bwd", code, P(dout), P(x), P(res), P(gamma), P(mean), P(rstd), P(dx), P(dres),
              P(gamma_grad), P(beta_grad), P(bias_grad), P(w), w.numel() * 4, rows, H, float(p),
              int(seed) & (2**64 - 1), stream())
    return dx, dres


def colsum(x, ld, rows, N, out, accumulate=True):
    nbytes = _lib.query("vcg_colsum_ws_bytes", rows, N)
    w = ws(nbytes, x.device)
    _lib.call("vcg_colsum", dt_code(x.dtype), P(x), ld, rows, N, P(out), int(accumulate), P(w), w.numel() * 4,
              stream())


def attn_softmax_fwd(S, mask, P_out, Pd_out, B, nh, L, Lp, scale, p=0.0, seed=0):
    _lib.call("vcg_attn_softmax_fwd", dt_code(S.dtype), P(S), P(mask), P(P_out), P(Pd_out), B, nh, L, Lp,
              float(scale), float(p), int(seed) & (2**64 - 1), stream())


def attn_softmax_bwd(dPd, Pm, dS, Z, L, Lp, scale, p=0.0, seed=0):
    _lib.call("vcg_attn_softmax_bwd", dt_code(dPd.dtype), P(dPd), P(Pm), P(dS), Z, L, Lp, float(scale), float(p),
              int(seed) & (2**64 - 1), stream())


def bert_attn_fwd(qkv, mask, ctx, stats, B, nh, L, Lp, scale, p=0.0, seed=0, seq=None):
    """Fused attention forward (bf16): qkv [B*L(+pad), 3H] -> ctx [B*L, H]; stats [B*nh*128, 2] f32.
    seq (int32 [B+1]): packed sequences, rows seq[b] .. seq[b+1]-1 (L = the longest, mask = the packed rows' key
    flags; vcg_bert_attn_fwd_varlen)."""
    if seq is None:
        _lib.call("vcg_bert_attn_fwd", P(qkv), P(mask), P(ctx), P(stats), B, nh, L, Lp, float(scale), float(p),
                  int(seed) & (2**64 - 1), stream())
    else:
        _lib.call("vcg_bert_attn_fwd_varlen", P(qkv), P(mask), P(seq), P(ctx), P(stats), B, nh, L, Lp, float(scale),
                  float(p), int(seed) & (2**64 - 1), stream())


def bert_attn_bwd(qkv, dctx, ctx, mask, stats, dqkv, B, nh, L, Lp, scale, p=0.0, seed=0, seq=None):
    if seq is None:
        _lib.call("vcg_bert_attn_bwd", P(qkv), P(dctx), P(ctx), P(mask), P(stats), P(dqkv), B, nh, L, Lp, float(scale),
                  float(p), int(seed) & (2**64 - 1), stream())
    else:
        _lib.call("vcg_bert_attn_bwd_varlen", P(qkv), P(dctx), P(mask), P(seq), P(stats), P(dqkv), B, nh, L, Lp,
                  float(scale), float(p), int(seed) & (2**64 - 1), stream())


def tanh_bwd(dy, t):
    dx = torch.empty_like(dy)
    _lib.call("vcg_tanh_bwd", dt_code(dy.dtype), P(dy), P(t), P(dx), dy.numel(), stream())
    return dx


# ----------------------------------------------------------------------------- head / loss
def head_mlp_fwd(Vout, Lout, W, bias, B, T, hid, O):
    logits = torch.empty((B, O), dtype=torch.float32, device=Vout.device)
    prob = torch.empty((B, O), dtype=torch.float32, device=Vout.device)
    _lib.call("vcg_head_mlp_fwd", dt_code(Vout.dtype), P(Vout), P(Lout), P(W), P(bias), P(logits), P(prob), B, T,
              hid, O, stream())
    return logits, prob


def head_mlp_bwd(Vout, Lout, W, dlogits, dW, dbias, B, T, hid, O, relu_mask=True):
    dV = torch.empty_like(Vout)
    dL = torch.empty_like(Lout)
    _lib.call("vcg_head_mlp_bwd", dt_code(Vout.dtype), P(Vout), P(Lout), P(W), P(dlogits), P(dV), P(dL), P(dW),
              P(dbias), B, T, hid, O, int(relu_mask), stream())
    return dV, dL


def head_attn_fwd(Vout, Lout, query, key, value, proj, B, T, hid, n_head, p=0.0, seed=0):
    """SelfAttention head (two_stream.py:31-48) over cat([Vout [B*T,hid], Lout [B,hid]]) per window:
    logits / prob [B, O] fp32 and the f32 state the backward needs (vcg_head_attn_saved_floats)."""
    _chk(Vout, name="Vout")
    _chk(Lout, Vout.dtype, "Lout")
    assert Vout.numel() == B * T * hid and Lout.numel() == B * hid
    O = proj.weight.shape[0]
    for lin in (query, key, value, proj):
        _chk(lin.weight, torch.float32, "head weight")
    saved = torch.empty(_lib.query("vcg_head_attn_saved_floats", B, T, hid, n_head), dtype=torch.float32,
                        device=Vout.device)
    logits = torch.empty((B, O), dtype=torch.float32, device=Vout.device)
    prob = torch.empty((B, O), dtype=torch.float32, device=Vout.device)
    _lib.call("vcg_head_attn_fwd", dt_code(Vout.dtype), P(Vout), P(Lout), P(query.weight), P(query.bias),
              P(key.weight), P(key.bias), P(value.weight), P(value.bias), P(proj.weight), P(proj.bias), P(saved),
              saved.numel(), P(logits), P(prob), B, T, hid, n_head, O, float(p), int(seed) & (2**64 - 1), stream())
    return logits, prob, saved


def head_attn_bwd(saved, query, key, value, proj, dlogits, Vout, Lout, B, T, hid, n_head, p=0.0, seed=0,
                  relu_mask=True):
    """Backward of head_attn_fwd: returns the ReLU-masked gradients of Vout / Lout; accumulates the
    query / key / value / proj parameter gradients into their .grad (when they require grad)."""
    O = proj.weight.shape[0]
    dV = torch.empty_like(Vout)
    dL = torch.empty_like(Lout)
    w = torch.empty(_lib.query("vcg_head_attn_bwd_ws_floats", B, T, hid), dtype=torch.float32, device=Vout.device)

    def g(t):
        return P(t.grad) if t.requires_grad else None
    _lib.call("vcg_head_attn_bwd", dt_code(Vout.dtype), P(saved), P(query.weight), P(key.weight), P(value.weight),
              P(proj.weight), P(dlogits), P(dV), P(dL), g(query.weight), g(query.bias), g(key.weight), g(key.bias),
              g(value.weight), g(value.bias), g(proj.weight), g(proj.bias), P(w), w.numel(), B, T, hid, n_head, O,
              float(p), int(seed) & (2**64 - 1), int(relu_mask), stream())
    return dV, dL


def cross_entropy_fwd(logits, labels):
    B, C = logits.shape
    loss = torch.empty((), dtype=torch.float32, device=logits.device)
    _lib.call("vcg_cross_entropy_fwd", P(logits), P(labels), P(loss), B, C, stream())
    return loss


def cross_entropy_bwd(logits, labels, dloss):
    B, C = logits.shape
    dlogits = torch.empty_like(logits)
    _lib.call("vcg_cross_entropy_bwd", P(logits), P(labels), P(dloss), P(dlogits), B, C, stream())
    return dlogits


# ----------------------------------------------------------------------------- optimiser
def sumsq(x, out, workspace=None):
    if workspace is None:
        workspace = ws(_lib.query("vcg_sumsq_ws_bytes"), x.device)
    _lib.call("vcg_sumsq", P(x), x.numel(), P(workspace), P(out), stream())
    return workspace


def adamw(p, g, m, v, wd_flags, flag_shift, lr, beta1, beta2, eps, wd, step, sumsq_dev=None, max_norm=1.0,
          grad_scale=1.0, shadow=None):
    import math
    bc1 = 1.0 - beta1 ** step
    bc2 = 1.0 - beta2 ** step
    step_size = lr / bc1
    bc2_sqrt = math.sqrt(bc2)
    _lib.call("vcg_adamw", P(p), P(g), P(m), P(v), P(wd_flags), flag_shift, p.numel(), float(lr), float(beta1),
              float(beta2), float(eps), float(wd), float(step_size), float(bc2_sqrt), P(sumsq_dev), float(max_norm),
              float(grad_scale), P(shadow), stream())


# ----------------------------------------------------------------------------- synthetic data
def synth(out, kind, key, a, b):
    _lib.call("vcg_synth", int(kind), P(out), out.numel(), int(key) & (2**64 - 1), float(a), float(b), stream())
    return out
