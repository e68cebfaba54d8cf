"""Single-node launcher: ``python -m pytorch_distributedtraining_amd.launch --nproc-per-node N script.py ...``

torchrun-compatible environment for every rank (RANK, LOCAL_RANK, WORLD_SIZE, LOCAL_WORLD_SIZE,
MASTER_ADDR=127.0.0.1, MASTER_PORT=<free port>, TORCHELASTIC_RESTART_COUNT), one process per GPU,
failure detection (the first rank that dies takes the group down: SIGTERM, then SIGKILL after a grace
period -- no hung survivors) and ``--max-restarts`` elastic-style restarts.
Children get ``--local-rank`` only with ``--use-local-rank-arg`` (the reference script parses
``--local_rank`` and reads LOCAL_RANK from the env, Stoke-DDP.py:153,166; ``parse_local_rank`` below
accepts both spellings).

Also exposes ``spawn(fn, nprocs, args)`` -- the mp.spawn pattern of Fairscale-DDP.py:122-132 with the
rendezvous env filled in (127.0.0.1 + free port).
"""
from __future__ import annotations

import argparse
import os
import signal
import subprocess
import sys
import time

from .utils.dist import find_free_port


def parse_local_rank(argv=None) -> int:
    """Accept --local-rank N / --local_rank N / --local-rank=N, else env LOCAL_RANK, else 0."""
    argv = sys.argv[1:] if argv is None else argv
    for i, a in enumerate(argv):
        for flag in ("--local-rank", "--local_rank"):
            if a == flag and i + 1 < len(argv):
                return int(argv[i + 1])
            if a.startswith(flag + "="):
                return int(a.split("=", 1)[1])
    v = os.environ.get("LOCAL_RANK")
    return int(v) if v not in (None, "", "None") else 0


def _worker_entry(local_rank, fn, nprocs, args, master_port):
    os.environ.update(RANK=str(local_rank), LOCAL_RANK=str(local_rank), WORLD_SIZE=str(nprocs),
                      LOCAL_WORLD_SIZE=str(nprocs), MASTER_ADDR="127.0.0.1", MASTER_PORT=master_port)
    fn(local_rank, *args)


def spawn(fn, nprocs: int, args=(), join: bool = True):
    """torch.multiprocessing.spawn with the env:// rendezvous prepared (fn(rank, *args))."""
    import torch.multiprocessing as mp

    port = os.environ.get("MASTER_PORT") or find_free_port()
    return mp.spawn(_worker_entry, args=(fn, nprocs, tuple(args), port), nprocs=nprocs, join=join)


def visible_gpu_count() -> int | None:
    """GPUs this process may use, counted WITHOUT touching HIP (the launcher forks ranks; a parent that has
    initialised the GPU must not): the first of HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES /
    CUDA_VISIBLE_DEVICES that is set, else the GPU nodes of the KFD topology in sysfs (CPU nodes report
    gfx_target_version 0).  None when neither says (then nothing is capped)."""
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            return len([x for x in v.split(",") if x.strip() not in ("", "-1")])
    root = "/sys/class/kfd/kfd/topology/nodes"
    try:
        n = 0
        for node in os.listdir(root):
            try:
                with open(os.path.join(root, node, "properties")) as f:
                    for line in f:
                        k, _, val = line.partition(" ")
                        if k == "gfx_target_version" and int(val) > 0:
                            n += 1
                            break
            except (OSError, ValueError):
                continue
        return n or None
    except OSError:
        return None


def _shared_gpu_queues(nproc: int) -> str | None:
    """GPU_MAX_HW_QUEUES for ranks that must share GPUs (more ranks than devices: one-GPU rehearsals), keeping
    <= 8 HIP hardware queues per GPU (each rank's compute, comm and copy streams) -- less queue contention,
    not a correctness requirement: since the xGMI collectives wait in ONE wave per rank, the world-4 one-GPU
    GPT-2 1.3B rehearsal passes with HIP's default 4 queues per rank
    (profiles/r4/r4_rehearsal_gpt2_fsdp_w4_q4_one_waiter.log).  One rank per GPU keeps HIP's default.  Counted
    by ``visible_gpu_count`` (no HIP initialisation in the launcher)."""
    ndev = visible_gpu_count()
    if ndev is None or not 0 < ndev < nproc:
        return None
    per_dev = -(-nproc // ndev)
    return str(max(1, 8 // per_dev))


def _launch_once(cmd, nproc, port, restart, use_local_rank_arg, grace_s):
    procs = []
    queues = None if "GPU_MAX_HW_QUEUES" in os.environ else _shared_gpu_queues(nproc)
    if queues is not None:
        print(f"[launch] {nproc} ranks share the GPUs: GPU_MAX_HW_QUEUES={queues} per rank", file=sys.stderr, flush=True)
    for r in range(nproc):
        env = dict(os.environ)
        env.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nproc), LOCAL_WORLD_SIZE=str(nproc),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   TORCHELASTIC_RESTART_COUNT=str(restart))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC for RCCL on this platform
        if queues is not None:
            env["GPU_MAX_HW_QUEUES"] = queues
        c = list(cmd)
        if use_local_rank_arg:
            c.append(f"--local-rank={r}")
        procs.append(subprocess.Popen(c, env=env, start_new_session=True))
    failed = None
    while True:
        alive = 0
        for r, p in enumerate(procs):
            rc = p.poll()
            if rc is None:
                alive += 1
            elif rc != 0 and failed is None:
                failed = (r, rc)
        if failed is not None or alive == 0:
            break
        time.sleep(0.2)
    if failed is not None:
        print(f"[launch] rank {failed[0]} exited with {failed[1]}; stopping the group", file=sys.stderr, flush=True)
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGTERM)
                except ProcessLookupError:
                    pass
        t0 = time.time()
        while time.time() - t0 < grace_s and any(p.poll() is None for p in procs):
            time.sleep(0.1)
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
        return failed[1] if failed[1] > 0 else 1
    return 0


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--nproc-per-node", "--nproc_per_node", type=int, default=1)
    ap.add_argument("--nnodes", type=int, default=1)
    ap.add_argument("--master-port", "--master_port", type=int, default=None)
    ap.add_argument("--max-restarts", "--max_restarts", type=int, default=0)
    ap.add_argument("--use-local-rank-arg", action="store_true")
    ap.add_argument("--grace-s", type=float, default=10.0)
    ap.add_argument("-m", dest="module", default=None, help="run a module instead of a script")
    ap.add_argument("script", nargs="?")
    ap.add_argument("script_args", nargs=argparse.REMAINDER)
    argv = list(sys.argv[1:] if argv is None else argv)
    if "-m" in argv:   # like python -m: everything after the module name belongs to the child
        i = argv.index("-m")
        a = ap.parse_args(argv[:i])
        a.module, a.script, a.script_args = argv[i + 1], None, argv[i + 2:]
    else:
        a = ap.parse_args(argv)
    if a.nnodes != 1:
        raise SystemExit("this launcher is single-node (use torch.distributed.run for multi-node rendezvous)")
    if a.module:
        cmd = [sys.executable, "-m", a.module] + ([a.script] if a.script else []) + a.script_args
    else:
        cmd = [sys.executable, a.script] + a.script_args
    rc = 1
    for restart in range(a.max_restarts + 1):
        port = a.master_port or int(find_free_port())
        rc = _launch_once(cmd, a.nproc_per_node, port, restart, a.use_local_rank_arg, a.grace_s)
        if rc == 0:
            break
        if restart < a.max_restarts:
            print(f"[launch] restarting group ({restart + 1}/{a.max_restarts})", file=sys.stderr, flush=True)
    return rc


if __name__ == "__main__":
    sys.exit(main())
