"""The single-node launcher: env contract, collective over gloo, failure propagation."""
import os
import subprocess
import sys
import textwrap

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(tmp_path, body, nproc=3):
    script = tmp_path / "w.py"
    script.write_text(textwrap.dedent(body))
    env = dict(os.environ, PYTHONPATH=REPO)
    return subprocess.run([sys.executable, "-m", "dnn_page_vectors_amd.launch", "--nproc", str(nproc), "--",
                           str(script)], env=env, cwd=str(tmp_path), capture_output=True, text=True, timeout=300)


def test_launch_allreduce(tmp_path):
    r = _run(tmp_path, """
        import os, torch, torch.distributed as dist
        assert os.environ["MASTER_ADDR"] == "127.0.0.1"
        dist.init_process_group("gloo")
        t = torch.tensor([float(dist.get_rank() + 1)])
        dist.all_reduce(t)
        open(f"out{dist.get_rank()}.txt", "w").write(str(float(t)))
        dist.destroy_process_group()
    """)
    assert r.returncode == 0, r.stderr
    for k in range(3):
        assert float((tmp_path / f"out{k}.txt").read_text()) == 6.0


def test_launch_propagates_failure(tmp_path):
    r = _run(tmp_path, """
        import os, sys, time
        if os.environ["RANK"] == "1":
            sys.exit(7)
        time.sleep(60)  # peers would hang; the launcher must terminate them
    """)
    assert r.returncode == 7


@pytest.mark.parametrize("W", [2, 4, 8])
def test_bench_spawns_ranks_for_gpus_n(W):
    """`python bench.py --gpus W` without torchrun: the bench itself spawns W rank processes
    (the driver's multi-GPU invocation); CPU dry run over gloo — one JSON line, n_gpus W, and
    the per-rank step-time spread the scaling run is read with."""
    import json

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "1"
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(W), "--dry-run", "--steps", "2",
                        "--warmup", "1"], env=env, cwd=REPO, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == W and out["config"]["parallelism"] == f"dp{W}"
    assert out["config"]["dist_backend"] == "gloo" and out["config"]["launch"] == "bench-spawn"
    assert out["steps"] == 2 and out["warmup"] == 1 and out["value"] > 0
    assert out["recall_candidates"] == W * 64 and out["dry_run"] is True
    pr = out["per_rank"]
    for k in ("step_ms_median_per_rank", "step_ms_min_per_rank", "step_ms_max_per_rank", "wall_ms_per_step_per_rank"):
        assert len(pr[k]) == W and all(v > 0 for v in pr[k]), (k, pr[k])
    sp = pr["step_ms_rank_spread"]
    assert sp["min"] <= sp["median"] <= sp["max"]
    assert pr["step_probe"] == "host clock" and pr["exposed_allreduce_ms_median_per_rank"] is None
    assert out["ranks_seen"] == W and out["graph_status"] == "off" and out["rccl_version"] is None
    # the driver's JSON contract
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in out, k
    assert out["higher_is_better"] is True and out["scaling"] == "weak"
    for k in ("model", "global_batch", "seq_len", "parallelism"):
        assert k in out["config"], k
    knobs = out["runtime_knobs"]  # every PAGEVEC_* and HIP knob in effect, with the HIP defaults
    assert "GPU_MAX_HW_QUEUES" in knobs and "HSA_ENABLE_IPC_MODE_LEGACY" in knobs


def test_bench_rejects_world_size_mismatch():
    """Under a torchrun-style environment a --gpus that differs from WORLD_SIZE is an error,
    never a silent single-GPU measurement."""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--dry-run", "--steps", "1",
                        "--warmup", "0"], env=env, cwd=REPO, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "world size 1 != --gpus 2" in (r.stderr + r.stdout)


def test_comm_micro_gloo_and_channel_sweep():
    """tools/comm_micro.py (the RCCL tuning table for the 8-GPU node) runs its collectives
    over gloo at W = 2, and --sweep-channels relaunches once per NCCL_MIN_NCHANNELS value."""
    import json

    env = dict(os.environ, PYTHONPATH=REPO, OMP_NUM_THREADS="1")
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "comm_micro.py"), "--sweep-channels", "2", "4",
                        "--nproc", "2", "--device", "cpu", "--scale", "0.002", "--iters", "1", "--warmup", "0",
                        "--models", "cdssm", "--bucket-mb", "1"], env=env, cwd=REPO, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    recs = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(recs) == 2 * 3  # per channel setting: 1 all-reduce + 2 all-gathers
    assert {x["env"].get("NCCL_MIN_NCHANNELS") for x in recs} == {"2", "4"}
    assert all(x["world"] == 2 and x["ms"] > 0 for x in recs)
