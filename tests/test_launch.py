"""The single-node launcher: env contract, collective over gloo, failure propagation."""
import os
import subprocess
import sys
import textwrap

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
