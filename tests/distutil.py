"""Launch tests/dist_worker.py on G ranks (torch.distributed.run, 127.0.0.1)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch(mode, cases, world, tmp, timeout=300):
    cf = os.path.join(tmp, "cases.json")
    with open(cf, "w") as f:
        json.dump(cases, f)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}",
           os.path.join(HERE, "dist_worker.py"), "--mode", mode, "--cases", cf, "--out", tmp]
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "2")
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env)
    assert p.returncode == 0, f"ranks failed (rc={p.returncode}):\n{p.stdout[-3000:]}\n{p.stderr[-3000:]}"
    return {c["name"]: [dict(np.load(os.path.join(tmp, f"{c['name']}_rank{r}.npz"))) for r in range(world)]
            for c in cases}


def assemble(parts, key="x"):
    n = sum(p["rows"].size for p in parts)
    out = np.zeros(n)
    for p in parts:
        out[p["rows"]] = p[key]
    return out
