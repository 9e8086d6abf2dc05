"""Rank launcher of the bench scripts (one process per GPU).

`python bench.py --gpus N` must measure N GPUs whether or not the caller
wrapped it in `torch.distributed.run`.  When N > 1 and no rank environment
is present, the calling process starts ONE fresh child,
`python -m torch.distributed.run --nnodes=1 --nproc-per-node N ... <script>
<same args>`, lets it write to the same stdout/stderr, and exits with its
return code.  This module imports neither torch nor the HIP library, so the
parent never touches the GPU (exec-ing or forking after GPU initialisation is
not allowed on this pool).  Under a launcher (WORLD_SIZE set) the world size
must equal --gpus: a mismatch is an error, never a silent 1-rank run.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys


def free_port() -> int:
    """A TCP port on 127.0.0.1 that is free at the time of the call."""
    s = socket.socket()
    try:
        s.bind(("127.0.0.1", 0))
        return int(s.getsockname()[1])
    finally:
        s.close()


def launcher_command(script: str, argv: list[str], nranks: int, port: int) -> list[str]:
    """The torch.distributed.run command that starts `nranks` ranks of
    `script` with the caller's arguments, rendezvous on 127.0.0.1."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nranks}",
            "--master-addr", "127.0.0.1", "--master-port", str(port), str(script)] + list(argv)


def world_from_env(env=None) -> int | None:
    env = os.environ if env is None else env
    w = env.get("WORLD_SIZE")
    return int(w) if w not in (None, "") else None


def ensure_ranks(gpus: int, script: str, argv: list[str], env=None, run=subprocess.run) -> int | None:
    """Make this process one of `gpus` ranks.

    * WORLD_SIZE set (a launcher started us): it must equal `gpus`
      (ValueError otherwise); returns None and the caller runs as that rank.
    * WORLD_SIZE unset and gpus <= 1: returns None (a single rank).
    * WORLD_SIZE unset and gpus > 1: runs `launcher_command` as a child
      process with the same environment and returns its exit code; the caller
      must exit with it without doing any work itself.
    """
    if gpus < 1:
        raise ValueError(f"--gpus must be >= 1, got {gpus}")
    env = dict(os.environ if env is None else env)
    world = world_from_env(env)
    if world is not None:
        if world != gpus:
            raise ValueError(f"WORLD_SIZE={world} but --gpus {gpus}: launch {gpus} ranks, or pass --gpus {world}")
        return None
    if gpus == 1:
        return None
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    cmd = launcher_command(script, argv, gpus, free_port())
    print(f"[launch] {gpus} ranks: {' '.join(cmd[1:])}", file=sys.stderr, flush=True)
    return int(run(cmd, env=env).returncode)
