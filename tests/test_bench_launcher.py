"""bench.py --gpus N launches N rank processes itself (no torch.distributed.run)
and reassembles one stream from exact-size shards: world size 2 on gloo, the
oracle as the per-shard codec (tests/bench_cpu_codec.py)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["PYTHONPATH"] = os.pathsep.join([ROOT, os.path.join(ROOT, "tests")])
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, cwd=ROOT,
                          capture_output=True, text=True, timeout=300)


@pytest.mark.parametrize("cfg", [2, 4])
@pytest.mark.parametrize("framed", [False, True], ids=["raw", "rm"])
def test_launcher_world2_gloo(cfg, framed):
    args = ["--gpus", "2", "--backend", "gloo", "--test-codec", "bench_cpu_codec", "--config", str(cfg),
            "--records", "1001", "--steps", "2", "--warmup", "1", "--gather-reps", "1"]
    if framed:
        args.append("--framed")
    p = _run(args)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout   # rank 0 alone prints the line
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "weak"
    assert d["config"]["records_per_gpu"] == 1001
    g = d["gather"]
    assert g["check"]["equal_to_1rank_encode"] is True
    assert g["check"]["checksum_ranks_agree"] is True
    assert g["stream_bytes"] > 0 and g["gather_inclusive_GiB_s"] > 0
    assert "send/recv" in g["collective"]   # gloo (CPU tensors) takes the exact send/recv path
    for leg in ("encode_only", "decode_only"):
        assert d[leg]["Mrec_s"] > 0


def test_world_size_mismatch_refused():
    p = _run(["--gpus", "2", "--test-codec", "bench_cpu_codec", "--backend", "gloo", "--records", "10"],
             env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0
    assert "WORLD_SIZE" in p.stderr


def test_launcher_ends_job_when_a_rank_dies():
    """Rank 1 exits 3 while rank 0 waits in a barrier: the launcher returns 3
    and kills rank 0 (it polls every rank, not rank 0 first)."""
    p = _run(["--gpus", "2", "--backend", "gloo", "--test-codec", "bench_fail_codec", "--config", "2",
              "--records", "100", "--steps", "1", "--warmup", "1"])
    assert p.returncode == 3, (p.returncode, p.stderr[-2000:])
    assert "rank 1 exits" in p.stderr
