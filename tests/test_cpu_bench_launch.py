"""`bench.py --gpus N` starts its own N rank processes (as the reference's DDP driver does with mp.spawn,
train_video_segment_ddp.py:599-608) when no launcher set WORLD_SIZE; the world it reports is N. CPU / gloo."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, extra_env=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(extra_env or {})
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, env=env, cwd=REPO,
                       capture_output=True, text=True, timeout=240)
    return p


def _line(out):
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_bench_gpus2_launches_two_ranks():
    p = _run(["--gpus", "2", "--launch-check"])
    assert p.returncode == 0, p.stderr[-3000:]
    j = _line(p.stdout)
    assert j["n_gpus"] == 2 and sorted(j["local_ranks"]) == [0, 1]
    # the self-validating fields a world > 1 line carries (the same ddp_evidence() as the GPU step)
    assert j["dist"] == {"backend": "gloo", "world_size": 2}
    assert j["params_consistent"] is True and j["params_max_abs_diff"] == 0.0
    ar = j["allreduce"]
    assert ar["buckets_per_step"] >= 2 and ar["wire_dtype"] == "fp32"
    assert ar["bytes_per_step"] >= 4 * (64 * 256 + 256 * 256 + 256 * 8)
    assert ar["exposed_ms_per_step_median"] >= 0.0


def test_bench_gpus4_launches_four_ranks():
    p = _run(["--gpus", "4", "--launch-check"])
    assert p.returncode == 0, p.stderr[-3000:]
    j = _line(p.stdout)
    assert j["n_gpus"] == 4 and j["dist"]["world_size"] == 4 and j["params_consistent"] is True


def test_bench_world_mismatch_fails():
    p = _run(["--gpus", "2", "--launch-check"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0 and "disagree" in (p.stderr + p.stdout)


def test_bench_long_video_rejects_multi_gpu():
    p = _run(["--gpus", "2", "--mode", "long_video"])
    assert p.returncode != 0 and "one-GPU" in (p.stderr + p.stdout)
