"""A/B of the 256 x 256-tile engine (igemm256.hip, VCG_G256=1) against the 128 x 128 engine on the step's
compute-bound GEMM shapes, in one process, interleaved rounds (HIP events): outputs compared bit for bit, times and
TF/s per engine. usage: python tools/bench_g256.py [rounds]"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "video-chapter-generation_amd"))
from vcg_hip import _lib, ops  # noqa: E402


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3  # us


def cases():
    dev, dt = "cuda", torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(1)
    out = []
    for name, M, N, K in (("bert ffn1 8192x3072x768", 8192, 3072, 768), ("bert ffn2 8192x768x3072", 8192, 768, 3072),
                          ("bert qkv 8192x2304x768", 8192, 2304, 768), ("l4 conv1 50176x512x2048", 50176, 512, 2048),
                          ("l3 conv3 200704x1024x256", 200704, 1024, 256), ("l4 conv3 50176x2048x512", 50176, 2048, 512),
                          ("square 8192^3", 8192, 8192, 8192)):
        A = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).to(dt)
        B = ((torch.rand(N, K, device=dev, generator=g) * 2 - 1) * 0.05).to(dt)
        C = torch.empty(M, N, dtype=dt, device=dev)
        out.append((name, 2.0 * M * N * K, lambda A=A, B=B, C=C, M=M, N=N, K=K: ops.gemm(A, B, M, N, K, K, K, out=C),
                    C))
    # (name, N, H, W, C, Cout, k, stride, pad, tsm)
    for name, N, H, W, Ci, Co, k, s, p, tsm in (("l2 conv2 3x3 128", 1024, 28, 28, 128, 128, 3, 1, 1, 0),
                                                 ("l3 conv2 3x3 256", 1024, 14, 14, 256, 256, 3, 1, 1, 0),
                                                 ("l4 conv2 3x3 512", 1024, 7, 7, 512, 512, 3, 1, 1, 0),
                                                 ("l3 conv1 1x1 1024 tsm", 1024, 14, 14, 1024, 256, 1, 1, 0, 16),
                                                 ("l4 conv1 1x1 2048 tsm", 1024, 7, 7, 2048, 512, 1, 1, 0, 16)):
        x = (torch.rand(N, H, W, Ci, device=dev, generator=g) * 2 - 1).to(dt)
        w = ((torch.rand(Co, k, k, Ci, device=dev, generator=g) * 2 - 1) * 0.05).to(dt)
        OH, OW = ops.conv_out_hw(H, W, k, k, s, p)
        y = torch.empty((N, OH, OW, Co), dtype=dt, device=dev)
        fold = Ci // 8 if tsm else 0
        out.append((name, 2.0 * N * OH * OW * Co * Ci * k * k,
                    lambda x=x, w=w, y=y, N=N, H=H, W=W, Ci=Ci, Co=Co, k=k, s=s, p=p, tsm=tsm, fold=fold:
                    ops.conv_fwd(x, w, N, H, W, Ci, Co, k, k, s, p, tsm, fold, out=y), y))
        M = N * OH * OW
        st = ops.stats_buffer(Co, M, dev)
        out.append((name + " +stats", 2.0 * M * Co * Ci * k * k,
                    lambda x=x, w=w, y=y, N=N, H=H, W=W, Ci=Ci, Co=Co, k=k, s=s, p=p, tsm=tsm, fold=fold, st=st:
                    ops.conv_fwd(x, w, N, H, W, Ci, Co, k, k, s, p, tsm, fold, stats=st, out=y), y, (st, M, Co)))
    return out


def finalize(st, M, C):
    out = [torch.empty(C, device="cuda") for _ in range(4)]
    ops.bn_finalize(st, st.shape[1], M, C, None, None, *out, None, None, 0.1, 1e-5)
    return out[0].double(), out[1].double()


def main():
    _lib.call("vcg_init", 0)
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    for case in cases():
        name, flops, fn, out = case[:4]
        stats = case[4] if len(case) > 4 else None
        modes = os.environ.get("G256_MODES", "0,1,2").split(",")
        res = {m: [] for m in modes}
        outs, fin = {}, {}
        for r in range(rounds):
            for mode in modes:
                os.environ["VCG_G256"] = mode
                out.zero_()
                res[mode].append(timeit(fn))
                if r == 0:
                    outs[mode] = out.clone()
                    if stats is not None:
                        fin[mode] = finalize(*stats)
        t0 = min(res["0"])
        line = f"{name:30s} 128-engine {t0:8.1f} us {flops / t0 / 1e6:7.1f} TF/s"
        for m in modes[1:]:
            t1 = min(res[m])
            same = torch.equal(outs["0"].view(torch.int16), outs[m].view(torch.int16))
            line += f" | G256={m} {t1:8.1f} us {flops / t1 / 1e6:7.1f} TF/s x{t0 / t1:5.2f} {'==' if same else '!='}"
            if stats is not None:
                (ma, ia), (mb, ib) = fin["0"], fin[m]
                line += f" stats d {((ma - mb).abs() * ia).max().item():.1e}/{((ia - ib).abs() / ia).max().item():.1e}"
        print(line, flush=True)
    os.environ["VCG_G256"] = "0"


if __name__ == "__main__":
    main()
