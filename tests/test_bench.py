"""The headline harness contract (``bench.py``): ``--gpus N`` starts N rank processes by itself
(no torchrun needed), the rank count must agree with a torchrun environment, and rank 0 prints
one JSON line whose ``value`` is the whole-job aggregate.  CPU: gloo ranks on the tiny model."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=300):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    env["CUDA_VISIBLE_DEVICES"] = ""          # CPU ranks (gloo) even where a GPU is visible
    env["HIP_VISIBLE_DEVICES"] = ""
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True,
                          text=True, timeout=timeout, env=env, cwd=ROOT)


def _json_lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


def test_bench_gpus2_spawns_two_ranks():
    r = _run(["--gpus", "2", "--model", "tiny", "--steps", "1", "--warmup", "0", "--no-score"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout                 # rank 0 only
    out = lines[0]
    assert out["n_gpus"] == 2
    assert out["comm"] == {"backend": "gloo", "world_size": 2, "oversubscribed": False}
    assert out["finite"] in (True, None)
    assert [p["rank"] for p in out["per_rank"]] == [0, 1]
    assert out["config"]["global_batch"] == 8
    # whole-job aggregate: 2 ranks x 4 images x 1 step over the slowest rank's time
    assert abs(out["value"] - 8 / (out["ms_per_step"] / 1e3)) / out["value"] < 0.01


def test_bench_world_size_mismatch_fails():
    r = _run(["--gpus", "2", "--model", "tiny", "--steps", "1", "--warmup", "0", "--no-score"],
             env_extra={"WORLD_SIZE": "1", "RANK": "0"}, timeout=120)
    assert r.returncode == 2
    assert "disagrees" in r.stderr


def test_bench_failing_rank_fails_the_job():
    # an unknown model raises in every rank: the launcher must exit non-zero, not hang
    r = _run(["--gpus", "2", "--model", "nope", "--steps", "1", "--warmup", "0", "--no-score"], timeout=120)
    assert r.returncode != 0
    assert not _json_lines(r.stdout)


def test_bench_live_supervised_topology():
    """tools/bench_live.py --gpus 2: front-end + 2 supervised workers (gloo on the CPU), both
    rooms drawn every round while the front-end scores"""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["CUDA_VISIBLE_DEVICES"] = ""
    env["HIP_VISIBLE_DEVICES"] = ""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "bench_live.py"), "--gpus", "2", "--model", "tiny",
                        "--players", "4", "--seconds", "3", "--idle-s", "1"], capture_output=True, text=True,
                       timeout=400, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    out = _json_lines(r.stdout)[-1]
    assert out["topology"] == "supervised" and out["n_gpus"] == 2
    assert out["devices"] == ["cpu:0", "cpu:1"] and not out["retired"]
    assert out["rounds"] >= 1 and out["images_per_s"] > 0 and out["requests"] > 0


def test_bench_oversubscribe_forces_gloo_and_refuses_nccl():
    r = _run(["--gpus", "2", "--oversubscribe", "--model", "tiny", "--steps", "1", "--warmup", "0", "--no-score"])
    assert r.returncode == 0, r.stderr[-3000:]
    out = _json_lines(r.stdout)[0]
    assert out["comm"] == {"backend": "gloo", "world_size": 2, "oversubscribed": True}
    assert len(out["per_rank"]) == 2
    r = _run(["--gpus", "2", "--oversubscribe", "--model", "tiny", "--steps", "1", "--warmup", "0", "--no-score"],
             env_extra={"CASSMANTLE_DIST_BACKEND": "nccl"}, timeout=120)
    assert r.returncode == 2 and "refused" in r.stderr


def test_bench_under_torchrun_four_ranks():
    """The driver's multi-GPU launch shape (torch.distributed.run, 127.0.0.1 rendezvous, one rank
    per device, bench.py reading RANK / WORLD_SIZE from the env): 4 gloo ranks on the CPU, one
    JSON line from rank 0 with the whole-job aggregate."""
    from cassmantle_amd.parallel.supervisor import free_port
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["CUDA_VISIBLE_DEVICES"] = ""
    env["HIP_VISIBLE_DEVICES"] = ""
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4",
                        "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.join(ROOT, "bench.py"),
                        "--gpus", "4", "--model", "tiny", "--steps", "1", "--warmup", "1", "--no-score"],
                       capture_output=True, text=True, timeout=400, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    out = lines[0]
    assert out["n_gpus"] == 4 and out["steps"] == 1 and out["warmup"] == 1
    assert out["comm"]["world_size"] == 4 and out["comm"]["backend"] == "gloo"
    assert out["config"]["parallelism"] == "dp4 (rooms)" and out["config"]["global_batch"] == 16
    assert [p["rank"] for p in out["per_rank"]] == [0, 1, 2, 3]
    assert abs(out["value"] - 16 / (out["ms_per_step"] / 1e3)) / out["value"] < 0.01
