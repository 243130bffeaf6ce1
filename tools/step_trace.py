"""Per-step wall times of the bench train step with allocator statistics (diagnosing run-to-run outliers):
python tools/step_trace.py [steps]. Prints one line per step: ms, num_alloc_retries, reserved GB."""
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "video-chapter-generation_amd"))
sys.path.insert(0, REPO)


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    from vcg_hip import _lib, synth
    from vcg_hip.build import build_two_stream
    from vcg_hip.functions import cross_entropy
    _lib.call("vcg_init", 0)
    dev = torch.device("cuda", 0)
    torch.manual_seed(123)
    model = build_two_stream(clip_frame_num=16, seed=123, device=dev, precision="bf16").train()

    class Cfg:
        weight_decay, learning_rate, betas = 0.01, 1e-5, (0.9, 0.95)
    opt = model.configure_optimizers(Cfg)
    frames, ids, mask, labels = synth.clip_batch(64, 16, 224, 224, 128, seed=123, device=dev)
    for i in range(steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        opt.zero_grad()
        logits, _ = model(frames, ids, mask)
        cross_entropy(logits, labels).backward()
        opt.clip_and_step(1.0)
        torch.cuda.synchronize()
        st = torch.cuda.memory_stats()
        print(f"step {i:3d} {1e3 * (time.perf_counter() - t0):8.2f} ms  retries {st.get('num_alloc_retries', 0)}  "
              f"reserved {torch.cuda.memory_reserved() / 2**30:6.1f} GB  peak {torch.cuda.max_memory_allocated() / 2**30:6.1f} GB",
              flush=True)


if __name__ == "__main__":
    main()
