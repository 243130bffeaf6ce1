"""TSM-ResNet-50 trunk on libvcg_hip: NHWC activations, BN statistics from the conv epilogue,
TSM shift fused into conv1's gather (fwd) and wgrad/dgrad (bwd).

Mirrors torchvision resnet50 + make_temporal_shift(place='blockres') exactly as the reference
builds it (model/vision/resnet50_tsm.py:15-19, ops/temporal_shift.py:104-146):
  stem conv7x7/2 -> bn -> relu -> maxpool3x3/2 ; layer1..4 Bottleneck v1.5 (stride on conv2) with
  conv1 = TemporalShift(conv1) ; avgpool ; fc = Identity.
Backward is written by hand (autograd never sees the kernels) and accumulates weight / BN gradients
straight into the parameters' flat fp32 .grad views.
"""
import os

import torch

from . import ops


def bn_mode(bn):
    """torch.nn.functional.batch_norm semantics for a BatchNorm2d module."""
    has_running = bn.running_mean is not None and bn.running_var is not None
    if bn.training:
        return "train" if (bn.track_running_stats and has_running) else "batch"
    return "running" if has_running else "batch"


class BNState:
    __slots__ = ("vec", "mean", "invstd", "scale", "shift", "mode", "count", "bn")

    def __init__(self, C, device, mode, count, bn):
        self.vec = torch.empty((4, C), dtype=torch.float32, device=device)
        self.mean, self.invstd, self.scale, self.shift = self.vec[0], self.vec[1], self.vec[2], self.vec[3]
        self.mode = mode
        self.count = count
        self.bn = bn


_WSTREAMS = {}  # device index -> the weight-gradient side stream


def _conv_shape(conv):
    KH, KW = conv.kernel_size
    return conv.out_channels, conv.in_channels, KH, KW, conv.stride[0], conv.padding[0]


def _tsm_info(conv1, Cin):
    """(conv module, T, fold) for a possibly TemporalShift-wrapped conv."""
    if hasattr(conv1, "net") and hasattr(conv1, "n_segment"):
        return conv1.net, conv1.n_segment, Cin // conv1.fold_div
    return conv1, 0, 0


class _ConvWeights:
    """bf16 GEMM operands of every trunk conv -- [Cout][KH][KW][Cpad] (fwd) and [Cin][KH][KW][Cout] (dgrad) --
    written by ONE vcg_weight_prep_multi launch per weight generation (flat.generation: once per optimizer
    step) instead of one launch per conv and use."""

    def __init__(self, net, flat, stem_cpad):
        self.flat = flat
        self.gen = None
        convs = [m for m in net.modules() if isinstance(m, torch.nn.Conv2d)]
        dev = convs[0].weight.device
        self.fwd, self.bwd = {}, {}
        desc = []
        self.stem_cpad = stem_cpad
        for conv in convs:
            Cout, Cin, KH, KW = conv.weight.shape
            stem = conv is net.conv1
            cpad = stem_cpad if stem else Cin
            if stem and cpad == 4:  # the pair-packed stem layout (ops.weight_prep pair_pad)
                pad = conv.padding[1]
                wf = torch.empty((Cout, KH, ops.pair_taps(KW, pad)[0], 8), dtype=torch.bfloat16, device=dev)
                mode = 2 + pad
            else:
                wf = torch.empty((Cout, KH, KW, cpad), dtype=torch.bfloat16, device=dev)
                mode = 0
            self.fwd[id(conv)] = wf
            desc.append([conv.weight.data_ptr(), wf.data_ptr(), Cout, Cin, KH, KW, cpad, mode])
            if not stem:  # the frames need no gradient
                wb = torch.empty((Cin, KH, KW, Cout), dtype=torch.bfloat16, device=dev)
                self.bwd[id(conv)] = wb
                desc.append([conv.weight.data_ptr(), wb.data_ptr(), Cout, Cin, KH, KW, Cin, 1])
        self.desc = torch.tensor(desc, dtype=torch.int64).to(dev)
        self.n = len(desc)
        self.ptrs = [conv.weight.data_ptr() for conv in convs]
        self.convs = convs

    def valid_for(self, net, flat, stem_cpad):
        return (flat is self.flat and stem_cpad == self.stem_cpad
                and [c.weight.data_ptr() for c in self.convs] == self.ptrs)

    def refresh(self):
        """Re-lay-out the weights after an optimizer step (one launch for all 53 convs). (Splitting it -- the stem's
        layout first, the rest on a side stream under the stem conv + max-pool -- measured neutral, round 2.)"""
        if self.gen == self.flat.generation:
            return
        self.gen = self.flat.generation
        ops.weight_prep_multi(self.desc, self.n)


class ResNetTrunk:
    staged = False  # forward() input is already the stem's NHWC layout [N, H, W, Cpad] (ops.window_frames_u8)
    # backward-path census (tests: the bf16 step must run the fused conv_dgrad_bwd engine everywhere)
    path_counts = {"fused": 0, "unfused": 0}
    # per-block path census (tests): a list to append to, or None. Forward entries ("fwd", C3, ds, {a2sum, y3_drop,
    # bn3_gemm}), backward entries ("bwd", C3, ds, {fold_wgrad, fold_dgrad}), in execution order
    census = None
    # False: run the bf16 backward through the unfused ops (conv_dgrad + bn_bwd_reduce / apply + tsm_unshift_add),
    # the reference path the fused conv_dgrad_bwd engine is checked against (tests/test_gpu_bf16_train.py)
    fused_bwd = True
    # bf16 backward: the weight gradients run on a side stream (one per device, _WSTREAMS), concurrently with the
    # input-gradient chain they branch off (each wgrad waits only for its dy); False: one stream
    wgrad_stream = True
    # forward of a layer's first bottleneck: the downsample conv on the side stream (False: inline)
    ds_stream = True
    # the first bottleneck of a layer: bn3's and the downsample BN's backward applies in one pass over g
    dual_bn_bwd = True
    # bf16 scoring forward (running-statistics BN, no autograd): bn3 folded into conv3 (1x1 GEMM with the BN scale in
    # the weight rows, the shift as bias, + identity, ReLU in the epilogue) -- no y3 tensor, no bn3 pass
    fold_eval = True
    # bf16 training backward: bn3's batch-statistics backward folded into conv3's two gradients (dy3 = A g + B y3 + C
    # is never stored: the input gradient is one GEMM over [g | y3], the weight gradient one GEMM with 2 C3 rows;
    # ops.conv_dgrad_bwd_bnfold / conv_wgrad_bnfold); False: the bn_bwd_apply pass
    bn_fold_bwd = True
    # ... for blocks with C3 <= this many channels (layers 1-3; layer 4's MFMA-bound conv3 gradients lose more to the
    # extra K than the pass costs: measured with the y3 drop, 78.6 vs 78.0 ms per step)
    bn_fold_max_c3 = 1024
    # ... with conv3's input a2 (C3 / 4 channels) as the second GEMM source instead of y3 (y3 = a2 w3^T: the input
    # gradient reads [g | a2] against [A w | w3^T diag(B) w3], the weight gradient is A (g^T a2) + B w3 (a2^T a2) + C
    # colsum(a2)); False: the y3 form
    bn_fold_a2 = True
    # ... and with both (non-first blocks): y3 is not stored at all -- conv3's forward GEMM keeps only the BN
    # statistics (ops.conv1x1_stats), the next block's conv1 dgrad reduces only sum g, and sum_gx comes from g^T a2
    # (ops.bn_bwd_sumgx_from_wgrad), which is also the weight gradient's first product; False: stored
    y3_drop = True
    # batch-statistics forward of a non-first bottleneck with C3 <= this many channels: bn3 + identity + ReLU as a
    # second pass of conv3's GEMM (scale folded into its weight rows, shift as bias; ops.conv1x1_bn_res_relu)
    # instead of reading y3 back in the bn_apply pass (0: off)
    bn3_gemm_max_c3 = 1024
    # bf16 batch statistics: the bn2 apply pass also returns colsum(a2) and a2^T a2 (ops.bn_apply_gram), from which
    # bn3's statistics follow where y3 is not stored (no statistics-only conv3 pass over a2) and the a2-form fold
    # takes its Gram term (no a2^T a2 GEMM in the backward); False: the conv3 statistics GEMM (tests compare both)
    gram_stats = True
    # the stem BN-backward sums from the pooled activation (ops.maxpool_bwd_bn_sums_pooled) instead of a pass over
    # the pre-pool conv output; False: the per-pixel pass (tests compare both)
    pooled_stem_sums = True
    # the stem's BN-backward apply and conv1 weight gradient as one pass (ops.stem_bwd_fused); False: the apply pass
    # writes dy0 and the im2col weight-gradient GEMM reads it (tests compare both)
    fused_stem_bwd = True
    # a y3-drop block's P = g^T a2 formed by the next block's streaming conv1 dgrad (layers 1-2); False: the weight-
    # gradient GEMM (tests compare both)
    dgrad_p = True
    # bn3's statistics, finalize and the GEMM pass's folded weight as one launch (ops.bn_finalize_from_gram) where the
    # Gram statistics apply; False: bn_stats_from_gram + bn_finalize + weight_fold (tests compare both)
    gram_fin = True

    def __init__(self, net, dtype):
        self.net = net
        self.dtype = dtype
        self._ws = None  # weight-gradient side stream of the running backward (_wside)
        self._pending = []  # (event, tensors) the side stream still reads (_hold)
        self.wc = None
        flat = getattr(net, "_vcg_flat", None)
        if dtype == torch.bfloat16 and flat is not None:
            wc = getattr(net, "_vcg_convw", None)
            if wc is None or not wc.valid_for(net, flat, ops.stem_cpad(dtype)):
                wc = _ConvWeights(net, flat, ops.stem_cpad(dtype))
                object.__setattr__(net, "_vcg_convw", wc)
            wc.refresh()
            self.wc = wc

    # ---------------------------------------------------------------- helpers
    def _wprep(self, conv, Cpad):
        if self.wc is not None:
            return self.wc.fwd[id(conv)]
        pair = self.dtype == torch.bfloat16 and Cpad == 4  # the stem (ops.stem_cpad)
        return ops.weight_prep(conv.weight.data, Cpad, self.dtype, pair_pad=conv.padding[1] if pair else None)

    def _wprep_t(self, conv, Cin):
        """[Cin][KH][KW][Cout]: the dgrad operand"""
        if self.wc is not None:
            return self.wc.bwd[id(conv)]
        return ops.weight_prep(conv.weight.data, Cin, self.dtype, transposed=True)

    def _drop_y3(self, blk, planes, need_grad):
        """This bottleneck's training forward keeps only bn3's statistics (see y3_drop)."""
        C3 = blk.conv3.out_channels
        if not need_grad:  # batch-statistics scoring: the GEMM pass is y3's only consumer
            return (ResNetTrunk.y3_drop and blk.downsample is None and self.dtype == torch.bfloat16
                    and C3 <= ResNetTrunk.bn3_gemm_max_c3 and C3 % 64 == 0
                    and planes % 64 == 0 and blk.conv3.stride[0] == 1 and bn_mode(blk.bn3) != "running")
        if blk is self.net.layer4[-1]:  # (its backward starts from the raw output gradient: bn3 needs y3)
            return False
        return (ResNetTrunk.y3_drop and need_grad and blk.downsample is None and ResNetTrunk.bn_fold_bwd
                and ResNetTrunk.bn_fold_a2 and ResNetTrunk.fused_bwd and self.dtype == torch.bfloat16
                and C3 <= ResNetTrunk.bn_fold_max_c3
                and C3 <= ResNetTrunk.bn3_gemm_max_c3 and C3 % 128 == 0 and planes >= 64
                and (planes & (planes - 1)) == 0 and blk.conv3.stride[0] == 1 and bn_mode(blk.bn3) != "running")

    def _conv_bn(self, x, conv, bn, N, H, W, C, tsm_T=0, tsm_fold=0, store=True):
        """conv -> BN statistics (+ running-stat update). store=False: a 1x1 conv keeps only the statistics (y =
        None, ops.conv1x1_stats)."""
        Cout, _, KH, KW, s, p = _conv_shape(conv)
        OH, OW = ops.conv_out_hw(H, W, KH, KW, s, p)
        M = N * OH * OW
        mode = bn_mode(bn)
        st = BNState(Cout, x.device, mode, M, bn)
        w = self._wprep(conv, C)
        if mode == "running":
            y = ops.conv_fwd(x, w, N, H, W, C, Cout, KH, KW, s, p, tsm_T, tsm_fold)
            ops.bn_eval_params(bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.eps, Cout, st.mean, st.invstd,
                               st.scale, st.shift)
        else:
            mt = ops.stats_tiles(M)
            stats = ops.stats_buffer(Cout, M, x.device)
            y = None
            if store or (KH, KW, s, p, tsm_fold) != (1, 1, 1, 0, 0) or not ops.conv1x1_stats(x.view(M, C), w, stats,
                                                                                               M, Cout, C):
                y = ops.conv_fwd(x, w, N, H, W, C, Cout, KH, KW, s, p, tsm_T, tsm_fold, stats=stats)
            self._finalize(stats, mt, M, Cout, bn, st)
        return y, st, OH, OW

    @staticmethod
    def _finalize(stats, mt, M, Cout, bn, st):
        upd = st.mode == "train"
        mom = bn.momentum if bn.momentum is not None else 0.1
        ops.bn_finalize(stats, mt, M, Cout, bn.weight, bn.bias, st.mean, st.invstd, st.scale, st.shift,
                        bn.running_mean if upd else None, bn.running_var if upd else None, mom, bn.eps)

    def _bn_from_gram(self, conv, bn, g64, M, C, fold=False):
        """BN state of conv's (1x1) output from its input's Gram matrix and column sums (ops.bn_stats_from_gram:
        y = x w^T is linear, so its batch mean / variance follow from x^T x and colsum(x) -- no pass over x or y).
        fold: also the conv weight folded by the new scale (bf16 [Cout, C], for conv1x1_bn_res_relu), else None."""
        Cout = conv.out_channels
        st = BNState(Cout, g64.device, bn_mode(bn), M, bn)
        w = self._wprep(conv, C).view(Cout, C)
        if ResNetTrunk.gram_fin and C <= 256 and C % 16 == 0:
            upd = st.mode == "train"
            w32 = conv.weight.data.view(Cout, C) if fold else None
            wf = torch.empty((Cout, C), dtype=torch.bfloat16, device=g64.device) if fold else None
            ops.bn_finalize_from_gram(g64, w, M, Cout, C, bn.weight, bn.bias, st.mean, st.invstd, st.scale, st.shift,
                                      bn.running_mean if upd else None, bn.running_var if upd else None,
                                      bn.momentum if bn.momentum is not None else 0.1, bn.eps, w32, wf)
            return st, wf
        stats = ops.stats_buffer(Cout, M, g64.device)
        ops.bn_stats_from_gram(g64, w, M, Cout, C, stats)
        self._finalize(stats, stats.shape[1], M, Cout, bn, st)
        return st, None

    # ---------------------------------------------------------------- forward
    def forward(self, x, need_grad):
        """x: [N, 3, H, W] fp32 frames ((b t) order), or (staged) the stem's NHWC input [N, H, W, Cpad] in the
        compute dtype. Returns (emb [N, 2048] fp32, saved)."""
        net, dt = self.net, self.dtype
        if self.staged:
            N, H, W, cpad = x.shape
            if x.dtype != dt or cpad != ops.stem_cpad(dt) or not x.is_contiguous():
                raise RuntimeError(f"staged frames must be contiguous NHWC [N,H,W,{ops.stem_cpad(dt)}] {dt}, "
                                   f"got {x.dtype} {tuple(x.shape)}")
            xs = x
        else:
            N, C0, H, W = x.shape
            cpad = ops.stem_cpad(dt)
            xs = ops.frames_to_nhwc(x.contiguous(), N, C0, H, W, cpad, dt)
        y0, b0, H1, W1 = self._conv_bn(xs, net.conv1, net.bn1, N, H, W, cpad)
        # bn1 + relu + maxpool in one pass (the activation never reaches HBM; the backward recomputes the ReLU
        # decision from y0)
        mp, idx = ops.bn_relu_maxpool(y0, b0.scale, b0.shift, N, H1, W1, 64)
        Hm, Wm = mp.shape[1], mp.shape[2]
        saved = {"stem": (xs, y0, mp, idx, b0, N, H, W, cpad, H1, W1)} if need_grad else None
        if not need_grad:
            del y0, idx
        h, Hc, Wc = mp, Hm, Wm
        self._fold_gen = None
        if ResNetTrunk.fold_eval and not need_grad and dt == torch.bfloat16:
            key = self._fold_key()
            old = getattr(net, "_vcg_fold_key", None)
            if old is None or old[0] != key:
                object.__setattr__(net, "_vcg_fold_key", (key, object()))
            self._fold_gen = net._vcg_fold_key[1]
        blocks = []
        for layer in (net.layer1, net.layer2, net.layer3, net.layer4):
            for blk in layer:
                h, rec, Hc, Wc = self._block_fwd(blk, h, N, Hc, Wc, need_grad)
                if need_grad:
                    blocks.append(rec)
        emb = ops.avgpool_fwd(h, N, Hc * Wc, h.shape[-1])
        if need_grad:
            saved["blocks"] = blocks
            saved["final"] = (N, Hc, Wc, h.shape[-1])
        return emb, saved

    def _block_fwd(self, blk, x, N, H, W, need_grad):
        Cin = x.shape[-1]
        conv1, T, fold = _tsm_info(blk.conv1, Cin)
        planes = conv1.out_channels
        if self._foldable(blk, x, need_grad):
            return self._block_fwd_folded(blk, x, conv1, T, fold, N, H, W)
        # the downsample branch (a layer's first block) depends only on x: its conv + BN statistics run on the side
        # stream, concurrently with conv1 -> conv2 -> conv3; the bn3 apply that adds it waits for it
        yd = bd = side = None
        cur = torch.cuda.current_stream() if x.is_cuda else None
        if blk.downsample is not None:
            side = self._wside(x.device) if self.ds_stream else None  # (an instance may turn it off)
            if side is not None:
                side.wait_stream(cur)
                with torch.cuda.stream(side):
                    yd, bd, _, _ = self._conv_bn(x, blk.downsample[0], blk.downsample[1], N, H, W, Cin)
                # (x stays referenced here until the join below; yd / bd come from the side stream's pool)
                yd.record_stream(cur)
                bd.vec.record_stream(cur)
        y1, b1, _, _ = self._conv_bn(x, conv1, blk.bn1, N, H, W, Cin, T, fold)
        a1 = ops.bn_apply(y1, b1.scale, b1.shift, planes, relu=True)
        y2, b2, H2, W2 = self._conv_bn(a1, blk.conv2, blk.bn2, N, H, W, planes)
        drop = self._drop_y3(blk, planes, need_grad)
        C3 = blk.conv3.out_channels
        a2sum = a2gram = g64 = None
        fold_a2 = (need_grad and ResNetTrunk.bn_fold_bwd and ResNetTrunk.bn_fold_a2 and ResNetTrunk.fused_bwd
                   and self.dtype == torch.bfloat16 and bn_mode(blk.bn3) != "running"
                   and C3 <= ResNetTrunk.bn_fold_max_c3 and planes <= 2048)
        if (fold_a2 or drop) and ResNetTrunk.gram_stats and planes in (64, 128, 256) and bn_mode(blk.bn3) != "running":
            # a2 with colsum(a2) and a2^T a2 from the bn2 apply pass: bn3's statistics follow from them (no conv3
            # statistics pass over a2 when y3 is not stored), and so does the Gram term of the a2-form backward fold
            a2, a2sum, a2gram, g64 = ops.bn_apply_gram(y2, b2.scale, b2.shift, planes, b2.mean, b2.invstd)
        elif fold_a2:
            # (the a2 form of the bn3 backward fold needs colsum(a2): written by the bn2 apply pass itself. A
            # separate column-sum pass on the side stream contended with conv3's GEMMs -- ~4 ms of kernel time per
            # step -- for the same step time, profiles/r04_a2sum_ab.txt)
            a2, a2sum = ops.bn_apply_colsum(y2, b2.scale, b2.shift, planes)
        else:
            a2 = ops.bn_apply(y2, b2.scale, b2.shift, planes, relu=True)
        wf = None
        if drop and a2gram is not None:
            # (a y3-drop block always takes the GEMM pass below: downsample-free, stride 1, batch statistics)
            b3, wf = self._bn_from_gram(blk.conv3, blk.bn3, g64, N * H2 * W2, planes,
                                        fold=self.dtype == torch.bfloat16 and C3 <= ResNetTrunk.bn3_gemm_max_c3)
            y3 = None
        else:
            y3, b3, _, _ = self._conv_bn(a2, blk.conv3, blk.bn3, N, H2, W2, planes, store=not drop)
        if not fold_a2:  # (the backward's a2-form fold reads these only where it applies)
            a2sum = a2gram = None
        r2 = None
        if blk.downsample is not None:
            if side is not None:
                cur.wait_stream(side)
            else:
                yd, bd, _, _ = self._conv_bn(x, blk.downsample[0], blk.downsample[1], N, H, W, Cin)
            # (bn3 + the downsample BN'd residual as a second conv3 GEMM pass measured neutral here, 805.3 vs 807.5
            # windows/s same box: the bn_apply pass over y3)
            out, obits = ops.bn_apply(y3, b3.scale, b3.shift, C3, relu=True, res=yd, rscale=bd.scale,
                                      rshift=bd.shift, bits=True)
        else:
            if (self.dtype == torch.bfloat16 and C3 <= ResNetTrunk.bn3_gemm_max_c3
                    and b3.mode != "running" and blk.conv3.stride[0] == 1):
                M = N * H2 * W2
                if wf is None:
                    wf = ops.weight_fold(blk.conv3.weight.data.view(C3, planes), b3.scale, self.dtype)
                r2 = ops.conv1x1_bn_res_relu(a2.view(M, planes), wf, b3.shift, x, M, C3, planes)
            if r2 is not None:
                out, obits = r2
            else:
                if y3 is None:  # (the GEMM pass did not apply: the conv output after all)
                    y3 = self._conv3_out(blk, a2, N, H2, W2, planes)
                out, obits = ops.bn_apply(y3, b3.scale, b3.shift, C3, relu=True, res=x, bits=True)
        if ResNetTrunk.census is not None:
            ResNetTrunk.census.append(("fwd", C3, blk.downsample is not None,
                                       {"a2sum": a2sum is not None, "y3_drop": y3 is None, "bn3_gemm": r2 is not None}))
        rec = None
        if need_grad:
            rec = dict(blk=blk, x=x, y1=y1, a1=a1, y2=y2, a2=a2, a2sum=a2sum, a2gram=a2gram, y3=y3, yd=yd, obits=obits, b1=b1, b2=b2, b3=b3,
                       bd=bd, N=N, H=H, W=W, H2=H2, W2=W2, Cin=Cin, planes=planes, C3=C3, T=T, fold=fold,
                       conv1=conv1)
        return out, rec, H2, W2

    def _conv3_out(self, blk, a2, N, H2, W2, planes):
        """conv3's output y3 recomputed from its input (where a stats-only forward dropped it)"""
        C3 = blk.conv3.out_channels
        return ops.conv_fwd(a2, self._wprep(blk.conv3, planes), N, H2, W2, planes, C3, 1, 1, 1, 0)

    def _y3(self, r):
        if r["y3"] is None:
            r["y3"] = self._conv3_out(r["blk"], r["a2"], r["N"], r["H2"], r["W2"], r["planes"])
        return r["y3"]

    def _foldable(self, blk, x, need_grad):
        """bf16 scoring forward with every BN of the block on running statistics and a 1x1 / stride-1 conv3."""
        if not (ResNetTrunk.fold_eval and not need_grad and self.dtype == torch.bfloat16 and x.is_cuda):
            return False
        bns = [blk.bn1, blk.bn2, blk.bn3] + ([blk.downsample[1]] if blk.downsample is not None else [])
        return all(bn_mode(b) == "running" for b in bns) and _conv_shape(blk.conv3)[2:] == (1, 1, 1, 0)

    def _fold_key(self):
        """What the folded weights depend on: the master weights (flat.generation moves with every optimizer step /
        in-place write) and the BN affine + running statistics (their tensors' version counters move with every
        load_state_dict / in-place write; a training forward's native running-stat update bumps the
        num_batches_tracked counters, which share one version counter when they are views of one buffer)."""
        flat = getattr(self.net, "_vcg_flat", None)
        v = 0
        for m in self.net.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                for t in (m.weight, m.bias, m.running_mean, m.running_var, m.num_batches_tracked):
                    if t is not None:
                        v += t._version
        return (flat.generation if flat is not None else None, v)

    def _fold(self, conv, bn, Cpad):
        """(folded bf16 GEMM weight [Cout][KH][KW][Cpad], bias), cached across scoring forwards until the weights
        or the BN state change (_fold_key)."""
        cache = self._fold_cache
        ent = cache.get(id(conv))
        if ent is None:
            ent = cache[id(conv)] = self._fold_new(conv, bn, Cpad)
        return ent

    def _fold_new(self, conv, bn, Cpad):
        """conv weight rows scaled by gamma * invstd of the running statistics, beta - mean * scale as bias (eval BN,
        test_video_segment_point.py:116-122)."""
        Cout, Cin, KH, KW, _, _ = _conv_shape(conv)
        st = BNState(Cout, conv.weight.device, "running", 0, bn)
        ops.bn_eval_params(bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.eps, Cout, st.mean, st.invstd,
                           st.scale, st.shift)
        w2 = conv.weight.data.view(Cout, Cin * KH * KW)
        if KH == KW == 1 and Cpad == Cin:
            return ops.weight_fold(w2, st.scale, self.dtype), st.shift
        wf = ops.weight_fold(w2, st.scale, torch.float32).view(Cout, Cin, KH, KW)
        return ops.weight_prep(wf, Cpad, self.dtype), st.shift

    @property
    def _fold_cache(self):
        c = getattr(self.net, "_vcg_fold_cache", None)
        if c is None or c[0] is not self._fold_gen:
            c = (self._fold_gen, {})
            object.__setattr__(self.net, "_vcg_fold_cache", c)
        return c[1]

    def _block_fwd_folded(self, blk, x, conv1, T, fold, N, H, W):
        """The bottleneck of the scoring forward with every BN folded into the conv before it: conv1 (+ TSM gather)
        and conv2 with bias + ReLU epilogues, the downsample conv with bias, conv3 as one GEMM with bias, the
        identity / downsample output as residual and ReLU -- no y tensors, no BN passes."""
        Cin = x.shape[-1]
        planes = conv1.out_channels
        w1, c1 = self._fold(conv1, blk.bn1, Cin)
        a1 = ops.conv_fwd_bias_act(x, w1, c1, ops.ACT_RELU, N, H, W, Cin, planes, 1, 1, 1, 0, T, fold)
        _, _, KH, KW, s, p = _conv_shape(blk.conv2)
        w2, c2 = self._fold(blk.conv2, blk.bn2, planes)
        a2 = ops.conv_fwd_bias_act(a1, w2, c2, ops.ACT_RELU, N, H, W, planes, planes, KH, KW, s, p)
        H2, W2 = a2.shape[1], a2.shape[2]
        C3 = blk.conv3.out_channels
        if blk.downsample is not None:
            cd = blk.downsample[0]
            Cd, _, KHd, KWd, sd, pd = _conv_shape(cd)
            wd, bd = self._fold(cd, blk.downsample[1], Cin)
            res = ops.conv_fwd_bias_act(x, wd, bd, ops.ACT_NONE, N, H, W, Cin, Cd, KHd, KWd, sd, pd)
        else:
            res = x
        w3, c3 = self._fold(blk.conv3, blk.bn3, planes)
        M = N * H2 * W2
        out = ops.gemm(a2.view(M, planes), w3, M, C3, planes, planes, planes, bias=c3,
                       act=ops.ACT_RELU | ops.ACT_FLAG_ROUND_PRE, residual=res.view(M, C3), ldr=C3)
        return out.view(N, H2, W2, C3), None, H2, W2

    # ---------------------------------------------------------------- backward
    def _bn_bwd(self, dout, y, st, C, mbits=None, affine=False):
        """BN backward of conv output y. The upstream gradient is masked by the ReLU that followed the BN:
        affine=True recomputes the decision fma(y, scale, shift) > 0 exactly as the forward made it;
        mbits are the forward's mask bits (bn3, where the residual joins before the ReLU)."""
        bn = st.bn
        dev = y.device
        sums = torch.empty((2, C), dtype=torch.float32, device=dev)
        need_affine = bn.weight is not None and bn.weight.requires_grad
        msc, msh = (st.scale, st.shift) if affine else (None, None)
        ops.bn_bwd_reduce(dout, None, y, st.mean, st.invstd, C, sums[0], sums[1],
                          bn.weight.grad if need_affine else None, bn.bias.grad if need_affine else None,
                          mbits=mbits, mscale=msc, mshift=msh)
        return ops.bn_bwd_apply(dout, None, y, st.mean, st.invstd, bn.weight, sums[0], sums[1], C,
                                train_stats=st.mode != "running", mbits=mbits, mscale=msc, mshift=msh)

    def _wside(self, dev):
        """The trunk's side stream (weight gradients in the backward, downsample branches in the forward; None: bf16
        fast engine only, otherwise everything on the current stream)."""
        if not (ResNetTrunk.fused_bwd and self.dtype == torch.bfloat16 and dev.type == "cuda"):
            return None
        key = dev.index if dev.index is not None else torch.cuda.current_device()
        st = _WSTREAMS.get(key)
        if st is None:
            st = _WSTREAMS[key] = torch.cuda.Stream(device=dev)
        return st

    def _async(self, fn, *tensors):
        """Run fn (weight-gradient kernels) on the side stream after everything issued so far on the current
        stream; the tensors it reads stay referenced until the side stream has used them (_hold)."""
        ws = self._ws
        if ws is None:
            return fn()
        ws.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(ws):
            out = fn()
        self._hold(tensors)
        return out

    def _hold(self, tensors):
        """Keep tensors that side-stream kernels read referenced until an event after those kernels has COMPLETED
        (or the backward's final join). Not record_stream: its deferred frees are reclaimed only as the allocator
        polls the side stream's events, and with the host running a step ahead and the side stream trailing, the
        pool grew to ~260 GB with a 1.2-1.4 s stall in some runs (bench.py "host" diagnostics)."""
        ev = torch.cuda.Event()
        ev.record(self._ws)
        self._pending.append((ev, [t for t in tensors if t is not None]))
        while self._pending and self._pending[0][0].query():  # completed on the GPU: safe to free
            self._pending.pop(0)

    def _report(self, hooks, params):
        """Tell the DDP reducer a group of parameters is final: on the side stream (after the current stream's
        work), where their last weight-gradient kernels ran."""
        if hooks is None:
            return
        if self._ws is None:
            return hooks(params)
        self._ws.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self._ws):
            hooks(params)

    def _ds_dgrad_side(self, cds, dyd, N, H, W, Cin, C3):
        """The downsample conv's input gradient on the side stream: (res, res_stride, event). 1x1 / stride 2 (bf16
        fused path): ONE dense GEMM over the output pixels, added by conv1's dgrad epilogue at the even (h, w) rows."""
        ws, cur = self._ws, torch.cuda.current_stream()
        ws.wait_stream(cur)
        with torch.cuda.stream(ws):
            if cds.stride[0] == 2:
                wt_ds = self._wprep_t(cds, Cin)
                Mo = dyd.numel() // C3
                # (a plain GEMM: the wide-tile engine, ops.ACT_FLAG_WIDE)
                res, res_stride = ops.gemm(dyd.view(Mo, C3), wt_ds.view(Cin, C3), Mo, Cin, C3, C3, C3,
                                           act=ops.ACT_FLAG_WIDE), 2
            else:
                res, res_stride = self._dgrad(cds, dyd, N, H, W), 1
            ev = torch.cuda.Event()
            ev.record(ws)
        self._hold((dyd,))
        res.record_stream(cur)  # (allocated from the side stream's pool, read by the current stream)
        return res, res_stride, ev

    def _wgrad(self, conv, x, dy, N, H, W, Cpad, T=0, fold=0):
        if not conv.weight.requires_grad:
            return
        Cout, Cin, KH, KW, s, p = _conv_shape(conv)
        self._async(lambda: ops.conv_wgrad(x, dy, conv.weight.grad, N, H, W, Cpad, Cin, Cout, KH, KW, s, p, T, fold,
                                           accumulate=True), x, dy)

    def _dgrad(self, conv, dy, N, H, W):
        Cout, Cin, KH, KW, s, p = _conv_shape(conv)
        wt = self._wprep_t(conv, Cin)
        return ops.conv_dgrad(dy, wt, N, H, W, Cin, Cout, KH, KW, s, p)

    def backward(self, d_emb, saved, hooks=None):
        """d_emb: [N, 2048] fp32. Accumulates all trunk parameter grads; `hooks(params)` is told
        when a block's gradients are final (DDP bucket all-reduce).

        bf16 (fast engine): every conv input gradient carries the next steps of the backward in its
        epilogue (ops.conv_dgrad_bwd): conv3 / conv2 dgrads emit the ReLU-masked gradient of bn2 / bn1
        and their BN-backward sums; conv1's dgrad applies the TSM adjoint, adds the residual-branch
        gradient and emits the previous block's masked output gradient g with the sums of its bn3 (and
        downsample BN). The separate reduce / TSM-combine passes remain only where the fused engine
        does not apply (fp32 parity mode)."""
        N, Hc, Wc, C = saved["final"]
        self._ws = self._wside(d_emb.device) if ResNetTrunk.wgrad_stream else None
        dout = ops.avgpool_bwd(d_emb.contiguous(), N, Hc * Wc, C, self.dtype).view(N, Hc, Wc, C)
        blocks = saved["blocks"]
        gin = None  # (g, sums3, sumsd): masked output gradient of the block + its BN sums (fused path)
        while blocks:
            rec = blocks.pop()  # frees the block's activations as soon as its backward is done
            prev = blocks[-1] if blocks else None
            dout, gin = self._block_bwd(rec, dout, gin, prev)
            self._report(hooks, list(rec["blk"].parameters()))
            del rec
        xs, y0, mp, idx, b0, N, H, W, cpad, H1, W1 = saved["stem"]
        sums0 = torch.zeros((2, 64), dtype=torch.float32, device=y0.device)
        dg0, db0 = self._bn_grads(b0)
        # the BN sums, then the BN-backward apply over (dout, idx, y0) with g recomputed -- no g tensor (1.34 ms vs
        # 0.77 + 0.88 ms for storing g and applying it, tools/bench_stem.py). The sums come from the pooled
        # activation mp (a window's gradient reaches its argmax pixel, whose activation is mp): dout and mp instead of
        # dout, idx and the 4x larger y0
        if ResNetTrunk.pooled_stem_sums:
            ops.maxpool_bwd_bn_sums_pooled(dout, mp, idx, y0, N, H1, W1, 64, b0.mean, b0.invstd, b0.scale, b0.shift,
                                           sums0, dg0, db0)
        else:
            ops.maxpool_bwd_bn(dout, idx, N, H1, W1, 64, y0, b0.mean, b0.invstd, b0.scale, b0.shift, sums0, dg0, db0,
                               store_g=False)
        conv1 = self.net.conv1
        if self._stem_fused_ok(conv1, xs, N, H, W, cpad, H1, W1):
            # the apply and the conv1 weight gradient in one pass: dy0 stays in LDS (ops.stem_bwd_fused)
            ops.stem_bwd_fused(dout, idx, y0, xs, N, H1, W1, b0.mean, b0.invstd, b0.scale, b0.shift, b0.bn.weight,
                               sums0, N * H1 * W1, b0.mode != "running", conv1.weight.grad)
        else:
            dy0 = ops.maxpool_bwd_bn_apply(dout, idx, N, H1, W1, 64, y0, b0.mean, b0.invstd, b0.scale, b0.shift,
                                           b0.bn.weight, sums0, N * H1 * W1, b0.mode != "running")
            self._wgrad(conv1, xs, dy0, N, H, W, cpad)
        self._report(hooks, list(self.net.conv1.parameters()) + list(self.net.bn1.parameters()))
        if self._ws is not None:  # every weight gradient is complete on the caller's stream
            torch.cuda.current_stream().wait_stream(self._ws)
            self._pending.clear()  # (later reuse of these blocks is ordered after the wait)

    def _stem_fused_ok(self, conv1, xs, N, H, W, cpad, H1, W1):
        """ops.stem_bwd_fused applies: bf16 pair-packed frames (C = 4), the 7x7 / 2 / pad 3 stem, even conv-output
        height, width a multiple of 8 up to 112, a weight gradient to add to, every operand below 4 GB (32-bit buffer
        offsets: beyond ~2600 frames per GPU the apply pass + weight-gradient GEMM run instead)."""
        w = conv1.weight
        return (ResNetTrunk.fused_stem_bwd and self.dtype == torch.bfloat16 and cpad == 4 and w.requires_grad
                and w.grad is not None and tuple(w.shape) == (64, 3, 7, 7) and conv1.stride == (2, 2)
                and conv1.padding == (3, 3) and H == 2 * H1 and W == 2 * W1 and H1 % 2 == 0 and W1 % 8 == 0
                and W1 <= 112 and ops.stem_bwd_fused_fits(N, H1, W1))

    def _bn_grads(self, st):
        bn = st.bn
        if bn.weight is not None and bn.weight.requires_grad:
            return bn.weight.grad, bn.bias.grad
        return None, None

    def _bn_apply_bwd(self, g, y, st, C, sums):
        """BN backward apply on an already-masked gradient g with precomputed sums (mask mode 0)."""
        return ops.bn_bwd_apply(g, None, y, st.mean, st.invstd, st.bn.weight, sums[0], sums[1], C,
                                train_stats=st.mode != "running")

    def _dgrad_bn(self, conv, dy, N, H, W, y, st, C):
        """Input gradient of `conv` followed by the backward of the BN (+ReLU) that produced its input:
        returns the gradient of that BN's conv output y."""
        Cout, Cin, KH, KW, s, p = _conv_shape(conv)
        wt = self._wprep_t(conv, Cin)
        sums = torch.empty((2, C), dtype=torch.float32, device=y.device)
        dg, db = self._bn_grads(st)
        g = None
        if ResNetTrunk.fused_bwd:
            g = ops.conv_dgrad_bwd(dy, wt, N, H, W, Cin, Cout, KH, KW, s, p, y=y, mean=st.mean, invstd=st.invstd,
                                   mscale=st.scale, mshift=st.shift, sums=sums, dgamma=dg, dbeta=db)
        ResNetTrunk.path_counts["unfused" if g is None else "fused"] += 1
        if g is None:
            da = ops.conv_dgrad(dy, wt, N, H, W, Cin, Cout, KH, KW, s, p)
            return self._bn_bwd(da, y, st, C, affine=True)
        return self._bn_apply_bwd(g, y, st, C, sums)

    def _can_fold(self, r, ds):
        """bn3's backward folds into conv3's gradients here (bf16 fused engine, batch statistics, stored conv3 input,
        layers up to bn_fold_max_c3 channels). A first bottleneck runs its downsample BN's apply pass on the side
        stream where there is one (dyd feeds only the downsample's gradients), inline otherwise: the same kernels
        either way, so the one-stream instrumented / profiled step runs the timed step's path."""
        blk, b3, C3, planes = r["blk"], r["b3"], r["C3"], r["planes"]
        if not (ResNetTrunk.bn_fold_bwd and ResNetTrunk.fused_bwd and self.dtype == torch.bfloat16):
            return False
        if b3.mode == "running" or r["a2"] is None or C3 > ResNetTrunk.bn_fold_max_c3 or C3 % 128 != 0:
            return False
        if blk.conv3.stride[0] != 1 or planes < 64 or (planes & (planes - 1)) != 0:
            return False
        return not ds or r["bd"].mode != "running"

    def _fold_conv3(self, r, g, sums3):
        """conv3's weight gradient with bn3's batch-statistics backward folded in (side stream): dW = A (g^T a2) +
        B (y3^T a2) + C colsum(a2) as one GEMM with 2 C3 rows. False where the engine does not apply."""
        blk = r["blk"]
        if not blk.conv3.weight.requires_grad:
            return True
        N, H2, W2, planes, C3 = r["N"], r["H2"], r["W2"], r["planes"], r["C3"]
        b3, a2, y3 = r["b3"], r["a2"], r["y3"]
        M = N * H2 * W2

        a2s = r.get("a2sum")
        if a2s is not None:  # the a2 form: g^T a2 and a2^T a2 (plain weight-gradient GEMMs), combined per row
            Pg0 = r.get("Pg")

            G0 = r.get("a2gram")

            def wfn():
                G = G0
                if G is None:
                    G = torch.empty((planes, planes, 1, 1), dtype=torch.float32, device=a2.device)
                    ops.conv_wgrad(a2, a2, G, N, H2, W2, planes, planes, planes, 1, 1, 1, 0, accumulate=False)
                Pg = Pg0
                if Pg is None:
                    Pg = torch.empty((C3, planes, 1, 1), dtype=torch.float32, device=a2.device)
                    ops.conv_wgrad(a2, g, Pg, N, H2, W2, planes, planes, C3, 1, 1, 1, 0, accumulate=False)
                ops.bn_bwd_fold_wgrad_a2(Pg.view(C3, planes), G.view(planes, planes),
                                         blk.conv3.weight.data.view(C3, planes), C3, planes, b3.mean, b3.invstd,
                                         b3.bn.weight, sums3[0], sums3[1], M, a2s,
                                         blk.conv3.weight.grad.view(C3, planes))
                return True
            return self._async(wfn, a2, g, sums3, a2s, Pg0, G0)

        def wfn():
            cs = torch.empty(planes, dtype=torch.float32, device=a2.device)
            ops.colsum(a2.view(M, planes), planes, M, planes, cs, accumulate=False)
            return ops.conv_wgrad_bnfold(a2, g, y3, b3.mean, b3.invstd, b3.bn.weight, sums3[0], sums3[1], M, cs,
                                         blk.conv3.weight.grad, N, H2, W2, planes, C3)
        return self._async(wfn, a2, g, y3, sums3)

    def _dgrad_bn_fold(self, conv, g, y3, b3, sums3, N, H, W, y, st, C, C3, a2=None, a2sum=None):
        """_dgrad_bn of conv3 with bn3's backward folded in: one GEMM over [g | y3] against [A w | B w] (or, with
        a2sum = colsum(a2), over [g | a2] against [A w | w^T diag(B) w]) plus the constant column bias. None
        where the engine does not apply."""
        Cout, Cin, KH, KW, s, p = _conv_shape(conv)
        wt = self._wprep_t(conv, Cin)
        M = N * H * W
        if a2sum is not None:
            wfold, bias = ops.bn_bwd_fold_weights_a2(wt.view(Cin, C3), Cin, C3, b3.invstd, b3.bn.weight, sums3[0],
                                                     sums3[1], M, a2sum)
            src, Ky = a2, Cin
        else:
            wfold, bias = ops.bn_bwd_fold_weights(wt.view(Cin, C3), Cin, C3, b3.mean, b3.invstd, b3.bn.weight,
                                                  sums3[0], sums3[1], M)
            src, Ky = y3, C3
        sums = torch.empty((2, C), dtype=torch.float32, device=y.device)
        dg, db = self._bn_grads(st)
        g2 = ops.conv_dgrad_bwd_bnfold(g, src, wfold, bias, N, H, W, Cin, C3, y=y, mean=st.mean, invstd=st.invstd,
                                       mscale=st.scale, mshift=st.shift, sums=sums, dgamma=dg, dbeta=db, Ky=Ky)
        if g2 is None:
            return None
        ResNetTrunk.path_counts["fused"] += 1
        return self._bn_apply_bwd(g2, y, st, C, sums)

    def _block_bwd(self, r, dout, gin, prev):
        """Backward of one bottleneck. `gin` (fused path): (g, sums3, sumsd) = this block's ReLU-masked output
        gradient and its BN sums; else `dout` is the raw output gradient. `prev`: the record of the block
        whose output is this block's input (None: the max-pool). Returns (dout, gin) for `prev`."""
        blk = r["blk"]
        N, H, W, H2, W2 = r["N"], r["H"], r["W"], r["H2"], r["W2"]
        Cin, planes, C3, T, fold = r["Cin"], r["planes"], r["C3"], r["T"], r["fold"]
        obits = r["obits"]
        ds = blk.downsample is not None
        bnf = None  # bn3's backward folded into conv3's gradients: (g, sums3)
        if gin is not None:
            g, sums3, sumsd = gin
            b3, bd = r["b3"], r.get("bd")
            if r["y3"] is None and not ds:  # bn3's sum_gx from g^T a2 (the conv1 dgrad reduced only sum g)
                Pg = r.get("Pg")  # (formed by the next block's conv1 dgrad from its stored g tiles where it could)
                if Pg is None:
                    Pg = torch.empty((C3, planes, 1, 1), dtype=torch.float32, device=g.device)
                    ops.conv_wgrad(r["a2"], g, Pg, N, H2, W2, planes, planes, C3, 1, 1, 1, 0, accumulate=False)
                ops.bn_bwd_sumgx_from_wgrad(Pg.view(C3, planes), self._wprep(blk.conv3, planes), C3, planes, b3.mean,
                                            b3.invstd, sums3[0], sums3[1], self._bn_grads(b3)[0])
                r["Pg"] = Pg
            if self._can_fold(r, ds):
                bnf = (g, sums3)
                dy3 = dyd = None
                if ds:
                    # the downsample BN's apply pass on the side stream when its input gradient runs there too (dyd
                    # then feeds only side-stream kernels); inline otherwise, where the main stream reads dyd
                    def dyd_fn():
                        return self._bn_apply_bwd(g, r["yd"], bd, C3, sumsd)
                    if self._ws is not None and self.ds_stream:
                        dyd = self._async(dyd_fn, g, r["yd"], *sumsd)
                    else:
                        dyd = dyd_fn()
            elif ResNetTrunk.dual_bn_bwd and ds and b3.mode != "running" and bd.mode != "running":  # g read once
                dy3, dyd = ops.bn_bwd_apply_dual(g, r["y3"], b3.mean, b3.invstd, b3.bn.weight, sums3[0], sums3[1],
                                                 r["yd"], bd.mean, bd.invstd, bd.bn.weight, sumsd[0], sumsd[1], C3)
            else:
                dy3 = self._bn_apply_bwd(g, self._y3(r), b3, C3, sums3)
                dyd = self._bn_apply_bwd(g, r["yd"], bd, C3, sumsd) if ds else None
        else:
            g = torch.empty_like(dout)
            dy3 = self._bn_bwd_g(dout, self._y3(r), r["b3"], C3, obits, g)
            dyd = self._bn_bwd(dout, r["yd"], r["bd"], C3, mbits=obits) if ds else None
        # the downsample branch's input gradient needs only dyd: on the side stream ahead of the weight gradients,
        # joined (by its own event) just before conv1's fused dgrad adds it
        ds_res = None
        if ds and self._ws is not None and self.ds_stream:
            ds_res = self._ds_dgrad_side(blk.downsample[0], dyd, N, H, W, Cin, C3)
        if bnf is not None and not self._fold_conv3(r, *bnf):  # (the engine does not apply: the pass on dy3)
            dy3 = self._bn_apply_bwd(bnf[0], self._y3(r), r["b3"], C3, bnf[1])
            bnf = None
        if bnf is None:  # (with the fold, conv3's weight gradient went out with it)
            self._wgrad(blk.conv3, r["a2"], dy3, N, H2, W2, planes)
        dy2 = None
        if bnf is not None:
            dy2 = self._dgrad_bn_fold(blk.conv3, bnf[0], r["y3"], r["b3"], bnf[1], N, H2, W2, r["y2"], r["b2"], planes,
                                      C3, a2=r["a2"], a2sum=r.get("a2sum"))
            if dy2 is None:  # (the fused engine does not apply: the unfused pass, and conv3's dgrad on dy3)
                dy3 = self._bn_apply_bwd(bnf[0], self._y3(r), r["b3"], C3, bnf[1])
        if ResNetTrunk.census is not None:
            ResNetTrunk.census.append(("bwd", C3, ds, {"fold_wgrad": bnf is not None, "fold_dgrad": dy2 is not None,
                                                       "p_dgrad": bool(r.get("Pg_dgrad")),
                                                       "a2_form": bnf is not None and r.get("a2sum") is not None}))
        if dy2 is None:
            dy2 = self._dgrad_bn(blk.conv3, dy3, N, H2, W2, r["y2"], r["b2"], planes)
        del dy3
        self._wgrad(blk.conv2, r["a1"], dy2, N, H, W, planes)
        dy1 = self._dgrad_bn(blk.conv2, dy2, N, H, W, r["y1"], r["b1"], planes)
        del dy2
        self._wgrad(r["conv1"], r["x"], dy1, N, H, W, Cin, T, fold)
        res_stride = 1
        if ds and ds_res is not None:
            self._wgrad(blk.downsample[0], r["x"], dyd, N, H, W, Cin)
            res, res_stride, ev = ds_res
            torch.cuda.current_stream().wait_event(ev)
        elif ds:
            cds = blk.downsample[0]
            self._wgrad(cds, r["x"], dyd, N, H, W, Cin)
            if cds.stride[0] == 2 and self.dtype == torch.bfloat16 and ResNetTrunk.fused_bwd:
                # 1x1 / stride 2: only the even (h, w) inputs receive a gradient, so it is ONE dense GEMM over the
                # output pixels (no 3/4-zero rows), added by the conv1 dgrad epilogue at those rows (res_stride 2)
                wt_ds = self._wprep_t(cds, Cin)
                Mo = dyd.numel() // C3
                res = ops.gemm(dyd.view(Mo, C3), wt_ds.view(Cin, C3), Mo, Cin, C3, C3, C3, act=ops.ACT_FLAG_WIDE)
                res_stride = 2
            else:
                res = self._dgrad(cds, dyd, N, H, W)  # the downsample branch's input gradient
        else:
            res = g  # the identity branch: the block's masked output gradient
        # conv1 input gradient + TSM adjoint + residual branch; fused: also the previous block's mask and sums
        conv1 = r["conv1"]
        Cout1, Cin1, KH, KW, s, p = _conv_shape(conv1)
        wt = self._wprep_t(conv1, Cin1)
        kw = dict(tsm_T=T if fold else 0, tsm_fold=fold, res=res, res_stride=res_stride)
        sums3 = sumsd = None
        if prev is not None:
            # rows: sum g, sum g (y3 - mean3) invstd3, sum g (yd - meand) invstdd; the downsample BN's (sum g, sum gx)
            # are rows 0 and 2 (one gradient feeds both BatchNorms)
            s3 = torch.empty((3 if prev["blk"].downsample is not None else 2, Cin), dtype=torch.float32,
                             device=dy1.device)
            sums3 = s3[:2]
            dg, db = self._bn_grads(prev["b3"])
            kw.update(bits=prev["obits"], y=prev["y3"], mean=prev["b3"].mean, invstd=prev["b3"].invstd, sums=sums3,
                      dgamma=dg, dbeta=db)
            if prev["blk"].downsample is not None:
                sumsd = (s3[0], s3[2])
                dg2, db2 = self._bn_grads(prev["bd"])
                kw.update(y2=prev["yd"], mean2=prev["bd"].mean, invstd2=prev["bd"].invstd, sum_gx2=s3[2],
                          dgamma2=dg2, dbeta2=db2)
        pg = None
        if (ResNetTrunk.fused_bwd and ResNetTrunk.dgrad_p and prev is not None and prev["y3"] is None
                and prev["blk"].downsample is None and prev["a2"] is not None and prev["planes"] == 64
                and prev["a2"].numel() == N * H * W * prev["planes"]):
            # the previous block's P = g^T a2 (its bn3 sum_gx and conv3 weight gradient) from this dgrad's stored g
            # tiles instead of a weight-gradient GEMM that re-reads g and a2 (layer 1: the dgrad pays 110-245 us for
            # a 405 us GEMM; with layer 2's 128 columns it pays as much as it saves, tools/bench_dgrad_p.py)
            pg = torch.empty((Cin1, prev["planes"], 1, 1), dtype=torch.float32, device=dy1.device)
            out, done = ops.conv_dgrad_bwd(dy1, wt, N, H, W, Cin1, Cout1, KH, KW, s, p, a2=prev["a2"],
                                           pg=pg.view(Cin1, prev["planes"]), **kw)
            if done:
                prev["Pg"] = pg
                prev["Pg_dgrad"] = True
        else:
            out = ops.conv_dgrad_bwd(dy1, wt, N, H, W, Cin1, Cout1, KH, KW, s, p, **kw) if ResNetTrunk.fused_bwd else None
        ResNetTrunk.path_counts["unfused" if out is None else "fused"] += 1
        if ds:
            if out is None and res_stride == 2:  # unfused fallback: the full-grid downsample input gradient
                res = self._dgrad(blk.downsample[0], dyd, N, H, W)
            del dyd
        if out is not None:
            if prev is None:
                return out, None  # the max-pool's output gradient (no mask, no BN)
            return None, (out, sums3, sumsd)
        dxs = ops.conv_dgrad(dy1, wt, N, H, W, Cin1, Cout1, KH, KW, s, p)
        return ops.tsm_unshift_add(dxs, res, N, T if T else 1, H * W, Cin, fold), None

    def _bn_bwd_g(self, dout, y, st, C, mbits, gout):
        """bn3 backward from the raw output gradient (mask bits), also writing the masked gradient g."""
        bn = st.bn
        sums = torch.empty((2, C), dtype=torch.float32, device=y.device)
        dg, db = self._bn_grads(st)
        ops.bn_bwd_reduce(dout, None, y, st.mean, st.invstd, C, sums[0], sums[1], dg, db, mbits=mbits)
        return ops.bn_bwd_apply(dout, None, y, st.mean, st.invstd, bn.weight, sums[0], sums[1], C,
                                train_stats=st.mode != "running", mbits=mbits, gout=gout)
