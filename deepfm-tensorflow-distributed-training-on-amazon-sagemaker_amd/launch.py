"""Launcher with restart-on-failure: one process per GPU via torch.distributed.run,
rerun up to ``--max_restarts`` times when any rank fails (watchdog exit, killed rank, RCCL error);
each run resumes from ``model_dir``'s latest complete checkpoint (the Estimator restores it).

    python -m rocfm.launch --nproc 8 --max_restarts 2 -- --task_type train --model_dir /ckpt …

The child runs ``python -m torch.distributed.run --standalone --nproc-per-node N -m rocfm.cli …``
(rendezvous on 127.0.0.1).  The launcher itself never touches the GPU.
"""
from __future__ import annotations

import argparse
import os
import subprocess
import sys
import time


def build_cmd(nproc: int, cli_args, port: int):
    if nproc <= 1:
        return [sys.executable, "-m", "rocfm.cli"] + list(cli_args)
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
            "--master-addr", "127.0.0.1", "--master-port", str(port), "-m", "rocfm.cli"] + list(cli_args)


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    if "--" in argv:
        i = argv.index("--")
        own, cli = argv[:i], argv[i + 1:]
    else:
        own, cli = argv, []
    ap = argparse.ArgumentParser(prog="rocfm.launch")
    ap.add_argument("--nproc", type=int, default=1)
    ap.add_argument("--max_restarts", type=int, default=0)
    ap.add_argument("--port", type=int, default=29500)
    a = ap.parse_args(own)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    rc = 1
    for attempt in range(a.max_restarts + 1):
        if attempt:
            sys.stderr.write(f"[rocfm.launch] restart {attempt}/{a.max_restarts} (previous exit {rc}); "
                             "resuming from the latest checkpoint\n")
            env["ROCFM_RESTART"] = str(attempt)
            time.sleep(1.0)
        rc = subprocess.call(build_cmd(a.nproc, cli, a.port + attempt), env=env)
        if rc == 0:
            return 0
    return rc


if __name__ == "__main__":
    sys.exit(main())
