"""Process launcher: one worker process per GPU of this node.

The reference's ``distribute`` entry point is an empty file; the north star asks for a
launcher that places pipeline stages on the 8 GPUs of one node.  This launcher:
  * picks a free TCP port on 127.0.0.1 for the torch.distributed store (control plane bootstrap);
  * starts N children with RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR / MASTER_PORT and
    ``HSA_ENABLE_IPC_MODE_LEGACY=0`` (dmabuf IPC, required by RCCL on this ROCm);
  * monitors them: the first child to fail takes the whole job down (terminate -> kill after a
    grace period), so a dead stage never leaves the rest of the pipeline blocked on RCCL;
  * returns the job's exit code (0 only if every rank exited 0).
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time
from typing import Dict, List, Optional, Sequence


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def package_pythonpath(current: Optional[str] = None) -> str:
    """PYTHONPATH for child processes that import this package (``-m distributed_llm_inference``)
    however the parent was started (e.g. ``/path/to/distribute`` from another directory)."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    parts = [p for p in (current or "").split(os.pathsep) if p]
    return os.pathsep.join([root] + [p for p in parts if p != root])


def launch(nproc: int, argv: Sequence[str], env: Optional[Dict[str, str]] = None,
           port: Optional[int] = None, grace_s: float = 10.0, poll_s: float = 0.2,
           gpus: Optional[Sequence[int]] = None) -> int:
    """Run ``python <argv...>`` ``nproc`` times with distributed env vars; returns exit code."""
    port = port or free_port()
    base = dict(os.environ)
    base.update(env or {})
    base.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    base["PYTHONPATH"] = package_pythonpath(base.get("PYTHONPATH"))
    base["MASTER_ADDR"] = "127.0.0.1"
    base["MASTER_PORT"] = str(port)
    base["WORLD_SIZE"] = str(nproc)
    base["LOCAL_WORLD_SIZE"] = str(nproc)
    procs: List[subprocess.Popen] = []
    for r in range(nproc):
        e = dict(base)
        e["RANK"] = str(r)
        e["LOCAL_RANK"] = str(gpus[r] if gpus else r)
        procs.append(subprocess.Popen([sys.executable] + list(argv), env=e))
    rc = 0
    try:
        while True:
            alive = 0
            for p in procs:
                code = p.poll()
                if code is None:
                    alive += 1
                elif code != 0 and rc == 0:
                    rc = code
            if rc != 0:
                _shutdown(procs, grace_s)
                break
            if alive == 0:
                break
            time.sleep(poll_s)
    except KeyboardInterrupt:
        _shutdown(procs, grace_s)
        rc = 130
    return rc


def _shutdown(procs: List[subprocess.Popen], grace_s: float) -> None:
    for p in procs:
        if p.poll() is None:
            p.send_signal(signal.SIGTERM)
    deadline = time.time() + grace_s
    for p in procs:
        try:
            p.wait(timeout=max(0.1, deadline - time.time()))
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
