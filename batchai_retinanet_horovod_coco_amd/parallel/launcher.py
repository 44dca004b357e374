"""``mxrun``: local multi-process launcher (the ``mpirun`` of ``training_job.json:7``).

Spawns N ranks of a command on this node with ``RANK / WORLD_SIZE / LOCAL_RANK /
LOCAL_WORLD_SIZE / MASTER_ADDR / MASTER_PORT`` (torch.distributed rendezvous over a TCP store on
127.0.0.1) plus ``OMPI_COMM_WORLD_*`` for mpirun-style scripts.  Output lines are prefixed with
``[rank]`` (like mpirun's ``--tag-output``); if any rank fails, the others are terminated and the
first non-zero exit code is returned.  Children are started with ``subprocess`` from a process
that has not touched the GPU (never exec'd over a GPU-initialised process).
"""
from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import threading
import time
from typing import List, Optional


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _pump(stream, rank: int, out, tag: bool):
    for line in iter(stream.readline, b""):
        txt = line.decode(errors="replace")
        out.write(("[{}] ".format(rank) + txt) if tag else txt)
        out.flush()


def launch(nproc: int, cmd: List[str], master_addr: str = "127.0.0.1", master_port: Optional[int] = None,
           tag_output: bool = True, env: Optional[dict] = None, timeout: Optional[float] = None,
           capture: bool = True) -> int:
    """Run ``cmd`` as ``nproc`` ranks; returns the first non-zero exit code (0 if all succeed).

    ``capture=False`` lets the children write straight to this process's stdout/stderr (no
    prefixing; used by ``bench.py --gpus N`` so rank 0's JSON line is the parent's output)."""
    port = master_port or free_port()
    procs, threads = [], []
    for r in range(nproc):
        e = dict(os.environ if env is None else env)
        e.update({"RANK": str(r), "WORLD_SIZE": str(nproc), "LOCAL_RANK": str(r), "LOCAL_WORLD_SIZE": str(nproc),
                  "MASTER_ADDR": master_addr, "MASTER_PORT": str(port), "OMPI_COMM_WORLD_RANK": str(r),
                  "OMPI_COMM_WORLD_SIZE": str(nproc), "OMPI_COMM_WORLD_LOCAL_RANK": str(r),
                  "OMPI_COMM_WORLD_LOCAL_SIZE": str(nproc), "MXR_CHILD": "1"})
        e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if not capture:
            procs.append(subprocess.Popen(cmd, env=e, start_new_session=True))
            continue
        p = subprocess.Popen(cmd, env=e, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, start_new_session=True)
        procs.append(p)
        t = threading.Thread(target=_pump, args=(p.stdout, r, sys.stdout, tag_output), daemon=True)
        t.start()
        threads.append(t)
    rc = 0
    t0 = time.time()
    try:
        alive = set(range(nproc))
        while alive:
            for r in list(alive):
                c = procs[r].poll()
                if c is not None:
                    alive.discard(r)
                    if c != 0 and rc == 0:
                        rc = c
                        for q in procs:
                            if q.poll() is None:
                                os.killpg(q.pid, signal.SIGTERM)
            if timeout is not None and time.time() - t0 > timeout:
                rc = rc or 124
                for q in procs:
                    if q.poll() is None:
                        os.killpg(q.pid, signal.SIGKILL)
                break
            time.sleep(0.05)
    except KeyboardInterrupt:
        for q in procs:
            if q.poll() is None:
                os.killpg(q.pid, signal.SIGTERM)
        rc = 130
    for t in threads:
        t.join(timeout=2)
    return rc


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="mxrun", description="Launch N local ranks (mpirun -np subset).")
    ap.add_argument("-np", "--np", dest="np", type=int, required=True)
    ap.add_argument("--master-addr", default="127.0.0.1")
    ap.add_argument("--master-port", type=int, default=None)
    ap.add_argument("--hostfile", default=None, help="only local hosts are supported")
    ap.add_argument("--no-tag-output", action="store_true")
    ap.add_argument("--timeout", type=float, default=None)
    ap.add_argument("cmd", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    if a.hostfile:
        with open(a.hostfile) as f:
            hosts = {l.split()[0] for l in f if l.strip() and not l.startswith("#")}
        if hosts - {"localhost", "127.0.0.1", socket.gethostname()}:
            raise SystemExit("mxrun: remote hosts are not supported (single-node launcher)")
    cmd = a.cmd[1:] if a.cmd and a.cmd[0] == "--" else a.cmd
    if not cmd:
        raise SystemExit("mxrun: no command given")
    return launch(a.np, cmd, a.master_addr, a.master_port, not a.no_tag_output, timeout=a.timeout)


if __name__ == "__main__":
    sys.exit(main())
