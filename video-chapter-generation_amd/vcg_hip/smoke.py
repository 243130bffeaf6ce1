"""__graft_entry__.smoke(): one tiny TwoStream train step on cuda:0 through libvcg_hip, checked
against the CPU oracle (oracle/, test infrastructure) on identical seeded weights and inputs."""
import os
import sys


def run_smoke():
    import torch

    from vcg_hip import _lib, synth
    from vcg_hip.build import build_two_stream
    from vcg_hip.functions import cross_entropy

    repo = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    if repo not in sys.path:
        sys.path.insert(0, repo)
    from oracle import model as om  # checker only

    if not torch.cuda.is_available():
        raise RuntimeError("smoke() needs an MI355X (cuda:0)")
    _lib.call("vcg_init", 0)
    B, T, HW, L = 2, 4, 112, 32
    model = build_two_stream(clip_frame_num=T, seed=123, device="cuda", dropout=0.0)
    model.train()
    frames, ids, mask, labels = synth.clip_batch(B, T, HW, HW, L, seed=123, device="cuda")
    logits, prob = model(frames, ids, mask)
    loss = cross_entropy(logits, labels)
    loss.backward()
    torch.cuda.synchronize()
    gsum = sum(float(p.grad.abs().sum()) for p in model.parameters())
    if not (torch.isfinite(loss).item() and gsum > 0):
        raise RuntimeError(f"smoke: bad loss {loss.item()} / grad sum {gsum}")

    # oracle on the same weights (the BN running stats of `model` were updated by its train step,
    # so compare with the oracle's train-mode forward from a CPU copy of the initial state)
    cpu = build_two_stream(clip_frame_num=T, seed=123, dropout=0.0)
    p = dict(cpu.state_dict())
    with torch.no_grad():
        ref_logits, _, _, _ = om.two_stream(p, frames.cpu(), ids.cpu(), mask.cpu(), bn_mode="train")
    d = (logits.detach().cpu() - ref_logits).abs().max().item()
    print(f"smoke: loss {loss.item():.6f}  max|logits - oracle| = {d:.3e}  grad|sum| = {gsum:.4e}")
    if d > 1e-3:
        raise RuntimeError(f"smoke: logits differ from the oracle by {d}")
