"""Multi-process test harness: N local processes on 127.0.0.1 over gloo (the reference's own
'cluster without a cluster' pattern, Fairscale-DDP.py:27,122-132), results returned via files."""
import os
import pickle
import socket
import tempfile
import traceback

import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _entry(rank, world, port, fn, args, outdir):
    import faulthandler
    faulthandler.enable()       # a native crash in a worker prints its Python stack instead of vanishing
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(2)
    try:
        # file rendezvous: no TCP port to race for when many suites spawn workers back to back
        dist.init_process_group("gloo", init_method="file://" + os.path.join(outdir, "rdzv"), rank=rank,
                                world_size=world)
        res = fn(rank, world, *args)
        err = None
    except Exception:
        res, err = None, traceback.format_exc()
    finally:
        if dist.is_initialized():
            try:
                dist.destroy_process_group()
            except Exception:
                pass
    with open(os.path.join(outdir, f"r{rank}.pkl"), "wb") as f:
        pickle.dump((res, err), f)
    # The result is on disk: leave without running C++ static destructors.  Under a loaded host (pytest -n 4)
    # a gloo background thread still joinable at interpreter teardown aborts the worker ("terminate called
    # without an active exception") and spawn reports SIGABRT for a run that had succeeded.
    import sys
    sys.stdout.flush()
    sys.stderr.flush()
    os._exit(0)


def run_workers(fn, world=2, *args, timeout=240):
    """Run fn(rank, world, *args) in `world` spawned processes; return the list of results."""
    with tempfile.TemporaryDirectory() as d:
        ctx = mp.start_processes(_entry, args=(world, _free_port(), fn, args, d), nprocs=world, join=False,
                                 start_method="spawn")
        import time
        deadline = time.time() + timeout
        # ProcessContext.join returns as soon as ONE process exits cleanly: keep joining until all are done
        while not ctx.join(max(0.0, deadline - time.time())):
            if time.time() >= deadline:
                break
        for p in ctx.processes:
            if p.is_alive():
                p.kill()
        out, errs = [], []
        for r in range(world):
            path = os.path.join(d, f"r{r}.pkl")
            if not os.path.exists(path):
                codes = [p.exitcode for p in ctx.processes]
                errs.append(f"rank {r} produced no result (crashed or timed out); exit codes {codes}")
                continue
            with open(path, "rb") as f:
                res, err = pickle.load(f)
            if err:
                errs.append(f"rank {r} failed:\n{err}")
            out.append(res)
        if errs:
            raise RuntimeError("\n".join(errs))
        return out


def assert_adam_close(sd1, sd2, lr=1e-3, steps=3, frac=0.995, zero_grad_slices=None):
    """States trained with Adam(W) at world 1 vs world N: bf16 gradients reduced in a different order can flip
    the sign of near-zero components, and Adam then moves them ~lr the other way each step.  The bulk must agree
    tightly; every element must stay within the 2 * lr * steps displacement (+ lr of slack).
    ``zero_grad_slices``: {key suffix: slice} of elements whose exact gradient is 0 (e.g. an attention key bias:
    softmax is invariant to a per-query shift, so sum_j dK_j = 0) -- their Adam updates are pure rounding noise
    and only the displacement bound applies to them."""
    import torch
    for k in sd1:
        a, b = sd1[k].float(), sd2[k].float()
        close = torch.isclose(a, b, atol=3e-3, rtol=3e-2)
        for suffix, sl in (zero_grad_slices or {}).items():
            if k.endswith(suffix):
                close = close.clone()
                close.view(-1)[sl] = True
        assert close.float().mean() > frac, (k, float(close.float().mean()))
        assert float((a - b).abs().max()) <= 2 * steps * lr + lr, (k, float((a - b).abs().max()))

