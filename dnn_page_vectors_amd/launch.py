"""Single-node process launcher: one process per GPU, torchrun env contract.

    python -m dnn_page_vectors_amd.launch --nproc 8 [--port P] -- script.py args...
    python -m dnn_page_vectors_amd.launch --nproc 8 -m dnn_page_vectors_amd train --preset mlp_xgpu --synthetic

Every child gets RANK / LOCAL_RANK / WORLD_SIZE / LOCAL_WORLD_SIZE / MASTER_ADDR=127.0.0.1 /
MASTER_PORT (a free port unless given) and ``HSA_ENABLE_IPC_MODE_LEGACY=0`` (dmabuf IPC,
required by RCCL on this driver).  Children are started as *new* processes (never exec'd
from a process that touched the GPU); the launcher itself never initialises HIP.  If any
rank fails, the remaining ranks are terminated (by PID) and the launcher exits with the
first non-zero status — a hung peer therefore cannot keep the job alive past the
collective timeout of the surviving ranks.
"""
from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import time
from typing import List, Optional, Sequence


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch(cmd: Sequence[str], nproc: int, port: Optional[int] = None, env: Optional[dict] = None,
           poll_s: float = 0.2) -> int:
    port = port or free_port()
    procs: List[subprocess.Popen] = []
    base = dict(os.environ if env is None else env)
    base.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    for r in range(nproc):
        e = dict(base, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nproc), LOCAL_WORLD_SIZE=str(nproc),
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen(list(cmd), env=e))
    status = 0
    try:
        alive = set(range(nproc))
        while alive:
            for r in list(alive):
                rc = procs[r].poll()
                if rc is None:
                    continue
                alive.discard(r)
                if rc != 0 and status == 0:
                    status = rc
                    for o in alive:
                        procs[o].send_signal(signal.SIGTERM)
            time.sleep(poll_s)
    except KeyboardInterrupt:
        for p in procs:
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
        status = 130
    finally:
        deadline = time.time() + 30
        for p in procs:
            try:
                p.wait(timeout=max(0.1, deadline - time.time()))
            except subprocess.TimeoutExpired:
                p.kill()
    return status


def main(argv: Optional[Sequence[str]] = None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--nproc", type=int, default=1)
    ap.add_argument("--port", type=int, default=0)
    ap.add_argument("-m", dest="module", default=None, help="run a module (like python -m)")
    ap.add_argument("rest", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    rest = list(a.rest)
    if rest and rest[0] == "--":
        rest = rest[1:]
    if a.module:
        cmd = [sys.executable, "-m", a.module] + rest
    elif rest:
        cmd = [sys.executable] + rest
    else:
        ap.error("nothing to launch")
    return launch(cmd, a.nproc, a.port or None)


if __name__ == "__main__":
    sys.exit(main())
