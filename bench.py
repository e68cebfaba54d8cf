#!/usr/bin/env python
"""Flagship benchmark: GPT-2 1.3B, FSDP full-shard, bf16, fused AdamW + global grad-norm clipping,
synthetic tokens (random-init weights), seq 1024, 96 sequences per GPU (weak scaling; the MI355X's
288 GB let the per-GPU batch grow -- larger GEMMs, the optimizer step and every FSDP all-gather /
reduce-scatter amortised over more tokens: 16 -> 32 sequences +4 % (r1_v5 logs), 32 -> 64 +2.8 % at a
132 GB peak, 126.3k -> 129.8k tokens/s; stock torch FSDP gains 3.9 % from the same change,
profiles/r2_flagship_microbatch.log; 64 -> 96 +1.3 % at 188 GB, profiles/r2_flagship_microbatch_64_96_128.log).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload gpt2-fsdp|gpt2-ddp|resnet50-ddp]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

Times exactly K optimizer steps bracketed by barrier + device synchronize, takes the MAX over ranks,
and prints ONE JSON line on rank 0 whose ``value`` is the whole-job throughput.
Metric/config follow BASELINE.json ("tokens/sec GPT-2-1.3B FSDP ... at 1/2/4/8 MI355X"; ResNet-50 DDP
samples/sec via --workload resnet50-ddp).  BASELINE.md publishes no reference number -> vs_baseline null.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

# MIOpen find / perf database for the ResNet-50 (batch 256, NHWC bf16) convolutions, recorded on MI355X
# (scripts/gpu_miopen.sh): without it the first step of a fresh box spends minutes in MIOpen's find.
os.environ.setdefault("MIOPEN_USER_DB_PATH",
                      os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuning", "miopen"))


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="gpt2-fsdp",
                    choices=["gpt2-fsdp", "gpt2-ddp", "resnet50-ddp", "llama3-fsdp", "swinir-stoke", "resnet18-cpu"])
    ap.add_argument("--model", default=None)
    ap.add_argument("--micro-batch", type=int, default=None)
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--grad-clip", type=float, default=1.0)
    ap.add_argument("--reshard", type=int, default=1, help="FSDP reshard after forward (FULL_SHARD)")
    ap.add_argument("--act-ckpt", type=int, default=0)
    ap.add_argument("--act-ckpt-policy", default=None, choices=["full", "selective"],
                    help="what a checkpointed layer recomputes: the whole block forward (full), or only norms / "
                         "attention forward / SwiGLU with the GEMM outputs kept (selective; Llama default)")
    ap.add_argument("--act-ckpt-layers", default="all",
                    help="with activation checkpointing: 'all', a layer count, or 'auto' = recompute only as many "
                         "layers as the HBM needs (sized after the first warm-up step)")
    ap.add_argument("--profile-steps", type=int, default=0)
    ap.add_argument("--resnet-graph", type=int, default=0,
                    help="resnet50-ddp (and the ResNet secondary): capture the whole DDP step in a HIP graph "
                         "(fwd, bwd, clip, fused AdamW; at N > 1 the bucket all-reduces too)")
    ap.add_argument("--secondary", type=int, default=1,
                    help="gpt2-fsdp: also measure BASELINE.json's ResNet-50 DDP metric at the same world size "
                         "(JSON 'secondary')")
    ap.add_argument("--secondary-micro-batch", type=int, default=None,
                    help="images per GPU of the secondary ResNet measurement (default 256)")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu: plumbing rehearsal of any workload on gloo (tiny --model / --micro-batch)")
    ap.add_argument("--overlap-probe", type=int, default=1,
                    help="world > 1: after timing, measure exposed vs communication-only time (untimed)")
    ap.add_argument("--rehearse-world", type=int, default=0,
                    help="REHEARSAL, never a headline: run this rank's step as rank --rehearse-rank of a world of "
                         "this size on ONE GPU over torch's 'fake' process group (collectives complete without "
                         "moving data): per-rank compute ms/step, shard sizes and peak memory at world W")
    ap.add_argument("--rehearse-rank", type=int, default=-1, help="rank to play (default: the last)")
    ap.add_argument("--loss", default="feat", choices=["feat", "mse"], help="swinir-stoke loss")
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32"], help="swinir-stoke precision")
    ap.add_argument("--graph", type=int, default=0,
                    help="gpt2-ddp / swinir-stoke: capture the whole training step (fwd, bwd, clip, fused AdamW; at "
                         "N > 1 over RCCL also the gradient collectives) in a HIP graph and replay it "
                         "(utils.graphs.GraphedStep / Trainer.graph)")
    ap.add_argument("--fp8", type=int, default=0,
                    help="gpt2/llama: run the transformer linears' GEMMs in fp8 (ops.fp8.fp8_autocast, delayed "
                         "scaling); reported with dtype 'fp8-linears' -- never the bf16 headline")
    return ap.parse_args()


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def self_launch(args) -> int | None:
    """``--gpus N`` without a torchrun environment: start N ranks of this script as child processes (one per
    GPU, env:// rendezvous on 127.0.0.1) -- the reference's own launch patterns (Stoke-DDP.py:2
    ``torch.distributed.launch --nproc_per_node``, Fairscale-DDP.py:125-132 ``mp.spawn``).  The parent never
    touches the GPU and never re-execs; it waits for the group and returns its exit code.  Returns None
    when this process is itself a rank (torchrun / our launcher set WORLD_SIZE)."""
    if "WORLD_SIZE" in os.environ:
        world = int(os.environ["WORLD_SIZE"])
        if world != args.gpus:
            log(f"[bench] --gpus {args.gpus} but WORLD_SIZE={world}: refusing to report a mislabelled run")
            return 2
        return None
    if args.gpus <= 1:
        return None
    from pytorch_distributedtraining_amd.launch import _launch_once
    from pytorch_distributedtraining_amd.utils.dist import find_free_port
    cmd = [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]
    return _launch_once(cmd, args.gpus, int(find_free_port()), 0, False, 10.0)


def main():
    args = parse()
    rc = self_launch(args)
    if rc is not None:
        sys.exit(rc)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.rehearse_world > 1:
        return rehearse(args)
    if args.workload == "resnet18-cpu" or args.device == "cpu":   # config 1 / CPU plumbing rehearsal
        dev = torch.device("cpu")
        if world > 1:
            dist.init_process_group("gloo")
        if args.device == "cpu":
            torch.set_num_threads(max(1, int(os.environ.get("OMP_NUM_THREADS", "2"))))
    else:
        # PDT_BENCH_BACKEND=gloo + PDT_XGMI=1 rehearses the multi-rank path on a box with fewer GPUs than
        # ranks (ranks share devices round-robin; device collectives on the xGMI kernels) -- a plumbing
        # check, not a measurement: RCCL (the default) needs one GPU per rank.
        backend = os.environ.get("PDT_BENCH_BACKEND", "nccl")
        ndev = torch.cuda.device_count()
        torch.cuda.set_device(local_rank % max(1, ndev))
        dev = torch.device("cuda", local_rank % max(1, ndev))
        if world > 1:
            dist.init_process_group(backend, device_id=dev if backend == "nccl" else None)
        from pytorch_distributedtraining_amd.ops import _lib
        _lib.require()  # fail loudly if the HIP kernels are missing
    from pytorch_distributedtraining_amd.parallel import Comm
    comm = Comm()

    torch.manual_seed(1234)
    if args.workload.startswith("gpt2") or args.workload.startswith("llama"):
        result = bench_gpt2(args, comm, dev, world, rank)
    elif args.workload == "swinir-stoke":
        result = bench_swinir(args, comm, dev, world, rank)
    else:
        result = bench_resnet(args, comm, dev, world, rank)
    result["topology"] = topology(comm, dev)
    if args.secondary and args.workload == "gpt2-fsdp":
        # BASELINE.json names TWO headline metrics (GPT-2-1.3B FSDP tokens/s and ResNet-50 DDP samples/s, both
        # "at 1/2/4/8"): every run also measures the second one at the SAME world size, so each point of the
        # driver's scaling curve records both.  Outside the primary's timed region; its setup and first step
        # are guarded phases (bench_resnet guarded=True): a failure on any rank skips it on every rank together
        # and the primary line is still printed.
        import copy
        import gc
        gc.collect()
        torch.cuda.empty_cache()
        try:
            a2 = copy.copy(args)
            a2.workload, a2.micro_batch, a2.steps, a2.warmup = "resnet50-ddp", args.secondary_micro_batch, 10, 3
            if dev.type == "cpu":
                a2.steps, a2.warmup = 1, 1
            sec = bench_resnet(a2, comm, dev, world, rank, guarded=True)
            result["secondary"] = {k: sec[k] for k in ("metric", "value", "unit", "n_gpus", "ms_per_step", "steps",
                                                       "warmup", "dtype", "config", "collectives_per_step",
                                                       "comm_bytes_per_step") if k in sec}
        except SecondarySkipped as e:   # every rank raised this together: no rank is left in a collective
            log(f"[bench] secondary ResNet-50 measurement skipped on every rank: {e}")
            result["secondary_error"] = str(e)[:200]
        except Exception as e:  # noqa: BLE001 - one rank: nobody to strand, keep the primary line
            if world > 1:
                raise
            log(f"[bench] secondary ResNet-50 measurement failed: {e!r}")
            result["secondary_error"] = f"{type(e).__name__}: {e}"[:200]
    if not headline_ok(result, args, dev, world):
        sys.exit(3)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def rehearse(args):
    """``--rehearse-world W``: one process on one GPU plays rank R of a world of W through torch's ``fake``
    process-group backend.  Every engine takes its multi-rank code path -- the nccl-style branches of ``Comm``
    (reduce_scatter_tensor with AVG, all_gather_into_tensor, all_reduce, barrier) with world-W shard shapes and
    bucket plans -- while the collectives themselves move no data.  The line reports per-rank compute time,
    collective counts / payload bytes per step and peak memory at world W.  It is a readiness rehearsal, NOT a
    measurement of scaling: its metric says so and it never carries a headline value."""
    import torch
    import torch.distributed as dist
    from torch.testing._internal.distributed.fake_pg import FakeStore

    world = args.rehearse_world
    rank = args.rehearse_rank if args.rehearse_rank >= 0 else world - 1
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("fake", rank=rank, world_size=world, store=FakeStore())
    # the fake group leaves outputs untouched: an FSDP all-gather would hand the forward uninitialised weights
    # (NaN loss -- and NaN / zero operands draw less power, so the GPU clocks up and the rehearsal reads ~16 %
    # fast, profiles/r6/r6d_fake_world8_rehearsal.jsonl).  Fill every output the way the real collective would
    # (this rank's payload in every slot / this rank's own chunk): real values, and the bytes a real
    # all-gather / reduce-scatter writes into its output.
    real_ag, real_rs = dist.all_gather_into_tensor, dist.reduce_scatter_tensor

    def all_gather_into_tensor(out, inp, group=None, async_op=False):
        w = real_ag(out, inp, group=group, async_op=async_op)
        out.view(world, -1).copy_(inp.reshape(1, -1).expand(world, -1))
        return w

    def reduce_scatter_tensor(out, inp, op=dist.ReduceOp.SUM, group=None, async_op=False):
        w = real_rs(out, inp, op=op, group=group, async_op=async_op)
        out.view(-1).copy_(inp.reshape(world, -1)[rank])
        return w
    dist.all_gather_into_tensor, dist.reduce_scatter_tensor = all_gather_into_tensor, reduce_scatter_tensor
    from pytorch_distributedtraining_amd.ops import _lib
    _lib.require()
    from pytorch_distributedtraining_amd.parallel import Comm
    comm = Comm(xgmi=False)
    args.overlap_probe, args.secondary, args.gpus = 0, 0, world
    torch.manual_seed(1234)
    if args.workload.startswith("gpt2") or args.workload.startswith("llama"):
        res = bench_gpt2(args, comm, dev, world, rank)
    elif args.workload == "swinir-stoke":
        res = bench_swinir(args, comm, dev, world, rank)
    else:
        res = bench_resnet(args, comm, dev, world, rank)
    out = {"metric": f"REHEARSAL per-rank compute ms/step at fake world {world} (rank {rank}, one GPU, collectives "
                     f"move no data) -- {res['metric'].split(' (whole node)')[0]} -- not a measurement",
           "value": res["ms_per_step"], "unit": "ms/step/rank", "higher_is_better": False, "rehearsal": True,
           "n_gpus": 1, "steps": args.steps, "warmup": args.warmup, "ms_per_step": res["ms_per_step"],
           "world": world, "rank": rank, "backend": comm.backend,
           **{k: res[k] for k in ("collectives_per_step", "comm_bytes_per_step", "peak_mem_gb", "dtype", "config")
              if k in res}}
    print(json.dumps(out), flush=True)
    dist.destroy_process_group()
    return 0


class SecondarySkipped(RuntimeError):
    """Raised on EVERY rank at the same agreement point when any rank failed a guarded phase."""


def agree(comm, dev, err, phase):
    """Phase boundary of a guarded measurement: every rank contributes whether it failed; all raise
    together, so a failure on one rank never leaves the others blocked in the next collective."""
    import torch
    flag = torch.tensor([0.0 if err is None else 1.0], device=dev)
    if comm.world_size > 1:
        comm.all_reduce(flag, "max")
    if float(flag.item()) > 0:
        raise SecondarySkipped(f"{phase}: " + (f"{type(err).__name__}: {err}" if err is not None else "failed on another rank"))


def headline_ok(result, args, dev, world) -> bool:
    """N > 1 on GPUs: print a headline only if the process group really spans N ranks on N distinct devices
    (a run whose ranks shared a GPU, or whose c10d world disagrees, would be a mislabelled scaling point).
    PDT_BENCH_REHEARSAL=1 (the one-GPU multi-rank plumbing rehearsal) prints it, marked as a rehearsal."""
    topo = result.get("topology", {})
    if dev.type != "cuda" or world <= 1:
        return True
    ok = topo.get("c10d_world") == world == args.gpus and topo.get("distinct_devices") == world
    if ok:
        return True
    if os.environ.get("PDT_BENCH_REHEARSAL") == "1":
        result["rehearsal"] = True
        result["metric"] += " [REHEARSAL: ranks share GPUs -- not a measurement]"
        return True
    log(f"[bench] refusing to print a headline: c10d_world={topo.get('c10d_world')} n_gpus={args.gpus} "
        f"WORLD_SIZE={world} distinct_devices={topo.get('distinct_devices')}")
    return False


def topology(comm, dev):
    """Proof of what ran: the c10d world size read back from the process group, and every rank's device
    (ordinal, PCI domain:bus:device, gfx arch) gathered to rank 0 -- N distinct bus ids = N distinct GPUs."""
    import torch
    import torch.distributed as dist
    me = {"rank": comm.rank, "host": os.uname().nodename}
    if dev.type == "cuda":
        p = torch.cuda.get_device_properties(dev)
        me.update(device=torch.cuda.current_device(),
                  pci=f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}", arch=p.gcnArchName)
    else:
        me.update(device="cpu")
    ranks = comm.all_gather_object(me) if comm.world_size > 1 else [me]
    pcis = {r.get("pci") for r in ranks if r.get("pci")}
    return {"c10d_world": dist.get_world_size() if dist.is_initialized() else 1,
            "c10d_backend": dist.get_backend() if dist.is_initialized() else None,
            "distinct_devices": len(pcis) if pcis else 0, "devices": ranks}


def timed_loop(step_fn, args, comm, dev):
    import torch

    class _NoSync:
        @staticmethod
        def synchronize(_dev=None):
            pass
    torch_cuda = torch.cuda if dev.type == "cuda" else _NoSync
    for i in range(args.warmup):
        step_fn()
        if i == 0:
            torch_cuda.synchronize(dev)
            log(f"[bench] warmup step 0 done")
    # per-shape kernel picks were timed per rank inside the warm-up; agree them over the engine's group here,
    # where every rank arrives together (ops/picks.py), so all ranks time the same kernels
    from pytorch_distributedtraining_amd.ops import picks
    picks.agree(comm)
    comm.barrier()
    torch_cuda.synchronize(dev)
    comm.reset_stats()
    if dev.type == "cuda":
        torch.cuda.reset_peak_memory_stats(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step_fn()
        if (i + 1) % 10 == 0:
            log(f"[bench] step {i + 1}/{args.steps}")
    torch_cuda.synchronize(dev)
    comm.barrier()
    torch_cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    # collectives issued by the engines inside the timed steps (the two barriers excluded)
    calls, nbytes = comm.stats["calls"], comm.stats["bytes"]
    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    comm.all_reduce(t, "max")
    timed_loop.comm = {"collectives_per_step": round(calls / args.steps, 2),
                       "comm_bytes_per_step": int(nbytes / args.steps)}
    if dev.type == "cuda":
        timed_loop.comm["peak_mem_gb"] = round(torch.cuda.max_memory_allocated(dev) / 1e9, 2)
    if comm.world_size > 1 and dev.type == "cuda" and args.overlap_probe:
        # diagnostics only, after the measurement: a failure here must not cost the run its JSON line
        try:
            timed_loop.comm.update(overlap_probe(step_fn, comm, dev, float(t.item()) * 1000 / args.steps))
        except Exception as e:  # noqa: BLE001
            log(f"[bench] overlap probe skipped: {type(e).__name__}: {e}")
            timed_loop.comm["overlap_probe_error"] = f"{type(e).__name__}: {e}"[:200]
    return float(t.item())


def overlap_probe(step_fn, comm, dev, step_ms):
    """Untimed, after the measurement: (1) one more step with every collective wait bracketed by events on
    the waiting stream -> exposed (non-overlapped) communication per step; (2) that step's collectives
    replayed back to back with no compute -> communication-only time; overlap = 1 - exposed / comm-only."""
    import torch
    from pytorch_distributedtraining_amd.parallel import comm as C
    comm.op_log = []
    C.start_wait_timing()
    step_fn()
    exposed = C.stop_wait_timing()
    ops, comm.op_log = comm.op_log, None
    bufs, err = [], None
    try:
        for op, n, dt, d in ops:
            kind = op.split(":")[0]
            if kind == "all_gather":
                bufs.append((kind, op, torch.empty(n, dtype=dt, device=d), torch.empty(n * comm.world_size, dtype=dt, device=d)))
            elif kind == "reduce_scatter":
                bufs.append((kind, op, torch.empty(n // comm.world_size, dtype=dt, device=d), torch.empty(n, dtype=dt, device=d)))
            else:
                bufs.append((kind, op, torch.zeros(n, dtype=dt, device=d), None))
    except RuntimeError as e:  # e.g. out of memory on one rank only
        err, bufs = e, []
    # every rank agrees before the replay, so a local failure skips the probe everywhere instead of
    # leaving the other ranks blocked in a collective this rank never enters
    flag = torch.tensor([0.0 if err is None else 1.0], device=dev)
    comm.all_reduce(flag, "max")
    if flag.item() > 0:
        raise RuntimeError(f"replay buffers unavailable on some rank ({err})")

    def replay():
        for kind, op, a, b in bufs:
            red = op.split(":")[1] if ":" in op else "sum"
            if kind == "all_gather":
                comm.all_gather(b, a)
            elif kind == "reduce_scatter":
                comm.reduce_scatter(a, b, "avg" if red == "avg" else "sum")
            elif kind == "all_reduce":
                comm.all_reduce(a, red)
            elif kind == "broadcast":
                comm.broadcast(a, 0)
            elif kind == "reduce":
                comm.reduce(a, 0, "sum")
    replay()
    torch.cuda.synchronize(dev)
    comm.barrier()
    t0 = time.perf_counter()
    for _ in range(3):
        replay()
    torch.cuda.synchronize(dev)
    only = (time.perf_counter() - t0) * 1000 / 3
    r = torch.tensor([exposed, only], dtype=torch.float64, device=dev)
    comm.all_reduce(r, "max")
    exposed, only = float(r[0]), float(r[1])
    log(f"[bench] comm: exposed {exposed:.2f} ms/step, comm-only {only:.2f} ms/step, step {step_ms:.1f} ms, "
        f"overlap {100 * max(0.0, 1 - exposed / only) if only > 0 else 0:.1f} %")
    return {"exposed_comm_ms": round(exposed, 3), "comm_only_ms": round(only, 3),
            "overlap_pct": round(100 * max(0.0, 1 - exposed / only), 1) if only > 0 else None}


def comm_fields(world):
    """Traffic of the engines per timed step, for the JSON line (zero collectives at world 1)."""
    return dict(n_ranks=world, **getattr(timed_loop, "comm", {}))


def bench_gpt2(args, comm, dev, world, rank):
    import torch
    from pytorch_distributedtraining_amd.models import build_gpt2
    from pytorch_distributedtraining_amd.optim import FusedAdamW, clip_grad_norm_
    from pytorch_distributedtraining_amd.parallel import FullyShardedDataParallel, MixedPrecision, ShardingStrategy

    fsdp = args.workload in ("gpt2-fsdp", "llama3-fsdp")
    llama = args.workload.startswith("llama")
    name = args.model or ("llama3-8b" if llama else "gpt2-1.3b" if fsdp else "gpt2-124m")
    # per-GPU micro-batch sized for 288 GB HBM: GPT-2 124M DDP 16 -> 64 sequences 700k -> 886k tokens/s
    # (profiles/r2_gpt2_124m_ddp_microbatch.log); GPT-2 1.3B FSDP 32 -> 64 +2.8 % (module docstring), 64 -> 96
    # +1.3 % at 188 GB peak (128: +2.0 % at 243 GB -- not taken, leaves < 50 GB headroom;
    # profiles/r2_flagship_microbatch_64_96_128.log); Llama-3 8B with selective recompute on all 32 layers 8 -> 16
    # sequences 22.9k -> 24.9k tokens/s at 182 GB peak (AdamW's fixed 39 ms/step amortised;
    # profiles/r5/r5_llama3_8b_ckpt_policy.jsonl); 16 -> 32 sequences 25.2k -> 26.3k tokens/s at 231 GB peak (24: 25.9k,
    # 206 GB; profiles/r6/r6e_microbatch_and_rehearsal.jsonl).  GPT-2 1.3B stays at 96: 112 / 128 sequences measured
    # +0.4 % / -0.2 % at 216 / 244 GB (same file)
    mb = args.micro_batch or (32 if llama else 96 if fsdp else 64)
    S = args.seq
    with torch.device(dev):
        if llama:
            from pytorch_distributedtraining_amd.models.llama import build_llama
            model = build_llama(name, max_seq_len=max(S, 2048), activation_checkpointing=bool(args.act_ckpt or 1),
                                checkpoint_policy=args.act_ckpt_policy or "selective")
        else:
            model = build_gpt2(name, n_positions=max(1024, S), activation_checkpointing=bool(args.act_ckpt))
    nparams = model.num_params()
    flops_tok = model.flops_per_token(S)                    # causal attention: the FLOPs the model needs
    flops_tok_full = model.flops_per_token(S, causal=False)  # every score counted (full-matrix convention)
    if fsdp:
        strat = ShardingStrategy.FULL_SHARD if args.reshard else ShardingStrategy.SHARD_GRAD_OP
        model = FullyShardedDataParallel(model, sharding_strategy=strat, mixed_precision=MixedPrecision(),
                                         comm=comm, device=dev, keep_low_precision_grads=True)
        params = model.flat_parameters()
        sharded = True
        par = f"fsdp{world}"
    else:
        from pytorch_distributedtraining_amd.parallel.ddp import DistributedDataParallel
        model = DistributedDataParallel(model, comm=comm, compute_dtype=torch.bfloat16)
        params = model.optimizer_parameters()
        sharded = False
        par = f"dp{world}"
    # world > 1: the bucket all-reduces are captured with the step (RCCL; DDP.prepare_capture)
    graph = bool(args.graph) and not fsdp and dev.type == "cuda" and (world == 1 or comm.backend == "nccl")
    opt = FusedAdamW(params, lr=1e-4, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1, capturable=graph)
    g = torch.Generator(device=dev)
    g.manual_seed(1000 + rank)
    vocab = (model.module if hasattr(model, "module") else model).config.vocab_size
    batches = [torch.randint(0, vocab, (mb, S + 1), device=dev, generator=g) for _ in range(4)]
    state = {"i": 0, "loss": None}
    inner = model.module if hasattr(model, "module") else model
    ckpt_on = bool(getattr(inner.config, "activation_checkpointing", False))
    if ckpt_on and args.act_ckpt_layers not in ("all", "auto"):
        inner.config.checkpoint_layers = int(args.act_ckpt_layers)

    def size_checkpointing():
        """After one fully checkpointed step: keep as many layers' activations as fit in 85 % of HBM
        (per-layer bytes estimated from the saved-tensor inventory of a block, x1.2 margin)."""
        c = inner.config
        L = getattr(c, "n_layers", getattr(c, "n_layer", 0))
        d = getattr(c, "dim", getattr(c, "n_embd", 0))
        ffn = getattr(c, "ffn_dim", 4 * d)
        qkv = (c.n_heads + 2 * c.n_kv_heads) * c.head_dim if hasattr(c, "n_kv_heads") else 3 * d
        per_tok = 2 * (5 * d + qkv + 3 * ffn) * 1.2          # bf16 tensors a non-recomputed block keeps
        extra = per_tok * mb * S - 2 * d * mb * S             # minus the input a checkpointed block keeps anyway
        free = 0.85 * torch.cuda.get_device_properties(dev).total_memory - torch.cuda.max_memory_allocated(dev)
        keep = max(0, min(L, int(free // max(extra, 1))))
        t = torch.tensor([float(keep)], device=dev)
        comm.all_reduce(t, "min")                             # same policy on every rank
        c.checkpoint_layers = L - int(t.item())
        log(f"[bench] activation checkpointing sized to HBM: {c.checkpoint_layers}/{L} layers recomputed")

    from pytorch_distributedtraining_amd.ops.fp8 import fp8_autocast

    def step():
        b = batches[state["i"] % len(batches)]
        state["i"] += 1
        with fp8_autocast(enabled=bool(args.fp8)):
            loss = model(b[:, :-1], labels=b[:, 1:])
        loss.backward()
        _, coef, found = clip_grad_norm_(params, args.grad_clip, comm=comm, sharded=sharded, apply=False)
        opt.step(grad_scale=coef)
        opt.zero_grad(set_to_none=True)
        state["loss"] = loss

    if graph:
        from pytorch_distributedtraining_amd.utils.graphs import GraphedStep
        static = batches[0].clone()

        def graph_body(b):
            opt.zero_grad(set_to_none=False)          # gradients keep their addresses across replays
            loss = model(b[:, :-1], labels=b[:, 1:])
            loss.backward()
            _, coef, _ = clip_grad_norm_(params, args.grad_clip, comm=comm, sharded=False, apply=False)
            opt.step(grad_scale=coef)
            return loss.detach()
        if world > 1:
            model.prepare_capture()
        graphed = GraphedStep(graph_body, static, warmup=2)

        def step():                                   # noqa: F811 - the graphed replacement
            b = batches[state["i"] % len(batches)]
            state["i"] += 1
            state["loss"] = graphed(b)
    if ckpt_on and args.act_ckpt_layers == "auto":
        # two fully checkpointed steps, the peak taken over the second: the first one also runs the once-per-shape
        # kernel timings (ops.linear / ops.blaslt choices), whose transient buffers would inflate the peak and
        # make the sizing recompute every layer
        step()
        torch.cuda.synchronize(dev)
        torch.cuda.reset_peak_memory_stats(dev)
        step()
        torch.cuda.synchronize(dev)
        size_checkpointing()
    dt = timed_loop(step, args, comm, dev)
    tokens = world * mb * S * args.steps
    tps = tokens / dt
    log(f"[bench] {name} params={nparams/1e9:.3f}B loss={float(state['loss'].item()):.4f} "
        f"step={1000*dt/args.steps:.1f}ms MFU(bf16 2.5PF/GPU, causal attention FLOPs)="
        f"{tps*flops_tok/world/2.5e15*100:.1f}% (full-matrix attention FLOPs: "
        f"{tps*flops_tok_full/world/2.5e15*100:.1f}%)")
    metric = "tokens/sec GPT-2-1.3B FSDP (whole node)" if fsdp and name == "gpt2-1.3b" else \
        f"tokens/sec {name} {'FSDP' if fsdp else 'DDP'} (whole node)"
    if llama:
        metric = f"tokens/sec {name} FSDP + act-ckpt (whole node)"
    return {"metric": metric, "value": round(tps, 2), "unit": "tokens/s",
            "n_gpus": world if dev.type == "cuda" else 0, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(1000 * dt / args.steps, 3), "higher_is_better": True,
            "scaling": "weak", **comm_fields(world), "vs_baseline": None,
            "dtype": "fp8-linears" if args.fp8 else "bf16", "data": "synthetic",
            "mfu": {"causal_attention_flops": round(tps * flops_tok / world / 2.5e15, 4),
                    "full_attention_flops": round(tps * flops_tok_full / world / 2.5e15, 4),
                    "peak": "2.5 PFLOP/s dense bf16 per GPU"},
            "config": {"model": name, "global_batch": world * mb, "seq_len": S, "parallelism": par,
                       "micro_batch_per_gpu": mb, "params": nparams, "hip_graph": graph, "sharding": "full_shard" if args.reshard else
                       "shard_grad_op", "optimizer": "fused AdamW + global-norm clip",
                       **({"act_ckpt_policy": getattr(inner.config, "checkpoint_policy", "full")} if ckpt_on else {}),
                       **({"act_ckpt_layers": inner.config.checkpoint_layers
                           if inner.config.checkpoint_layers is not None else
                           getattr(inner.config, "n_layers", getattr(inner.config, "n_layer", None))}
                          if ckpt_on else {})}}


def bench_resnet(args, comm, dev, world, rank, guarded=False):
    """``guarded`` (the secondary measurement after the GPT-2 headline): model / data are built and one local
    step (forward, backward under ``no_sync``, optimizer step -- no collective) runs before the timed loop,
    with an agreement of all ranks after each phase (``agree``), so an OOM or kernel error on one rank skips
    the measurement on every rank instead of blocking the others in a DDP collective."""
    import torch
    from pytorch_distributedtraining_amd.models.resnet import resnet50
    from pytorch_distributedtraining_amd.optim import FusedAdamW, clip_grad_norm_
    from pytorch_distributedtraining_amd.parallel.ddp import DistributedDataParallel

    cpu = dev.type == "cpu"
    fail_rank = int(os.environ.get("PDT_BENCH_SECONDARY_FAIL_RANK", "-1")) if guarded else -1
    if not cpu and os.environ.get("PDT_CONV_BENCHMARK", "1") == "1":
        # MIOpen find per conv shape in the first (untimed) step instead of its immediate-mode heuristic:
        # 7,133 -> 7,999 samples/s (profiles/r1_v9_miopen_modes.log; exhaustive search adds nothing)
        torch.backends.cudnn.benchmark = True
    mb = args.micro_batch or (16 if cpu else 256)
    # PDT_RESNET_AUTOCAST=0: the DDP bf16 compute copy instead of fp32 parameters under autocast (convs / fc on
    # bf16 parameters the fused AdamW epilogue rewrites from fp32 masters, channels_last inside the flat, batch
    # norms fp32).  Measured equal (8,624-8,728 vs 8,722 samples/s, profiles/r3_s4_resnet50_compute_copy_ab.log):
    # the ~250 weight-cast / fp32 gradient-add launches it removes are not on the critical path -- autocast kept
    autocast = cpu or os.environ.get("PDT_RESNET_AUTOCAST", "1") == "1"
    err = None
    try:   # phase 1 (local): module, inputs
        if cpu:
            from pytorch_distributedtraining_amd.models.resnet import resnet18
            model = resnet18().to(memory_format=torch.channels_last)
        else:
            model = resnet50().to(dev).to(memory_format=torch.channels_last)
        x = torch.randn(mb, 3, 224, 224, device=dev).to(memory_format=torch.channels_last)
        if not autocast:
            x = x.bfloat16()
        y = torch.randint(0, 1000, (mb,), device=dev)
    except Exception as e:  # noqa: BLE001
        if not guarded:
            raise
        err = e
    if guarded:
        agree(comm, dev, err, "build")
    # phase 2: the DDP wrap (startup broadcast: every rank is here), then one local step
    model = DistributedDataParallel(model, comm=comm, reduce_dtype=None if cpu else torch.bfloat16,
                                    compute_dtype=None if autocast else torch.bfloat16)
    params = model.optimizer_parameters()
    graph = bool(args.resnet_graph) and not cpu and (world == 1 or comm.backend == "nccl")
    opt = FusedAdamW(params, lr=1e-3, betas=(0.9, 0.99), eps=1e-8, weight_decay=1e-4, capturable=graph)
    crit = torch.nn.CrossEntropyLoss()

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=not cpu and autocast):
            loss = crit(model(x).float(), y)
        loss.backward()
        _, coef, _ = clip_grad_norm_(params, args.grad_clip, comm=comm, sharded=False, apply=False)
        opt.step(grad_scale=coef)
        opt.zero_grad(set_to_none=not graph)

    if guarded:
        try:
            if rank == fail_rank:
                raise RuntimeError("injected secondary failure (PDT_BENCH_SECONDARY_FAIL_RANK)")
            # no collective at all: gradient buckets held (no_sync), buffers not broadcast -- a local failure
            # here cannot strand a peer
            bb, model.broadcast_buffers = model.broadcast_buffers, False
            try:
                with model.no_sync():
                    step()
            finally:
                model.broadcast_buffers = bb
            if not cpu:
                torch.cuda.synchronize(dev)
        except Exception as e:  # noqa: BLE001
            err = e
        agree(comm, dev, err, "first step")

    if graph:
        from pytorch_distributedtraining_amd.utils.graphs import GraphedStep

        def body(xs, ys):
            opt.zero_grad(set_to_none=False)          # gradients keep their addresses across replays
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=autocast):
                loss = crit(model(xs).float(), ys)
            loss.backward()
            _, coef, _ = clip_grad_norm_(params, args.grad_clip, comm=comm, sharded=False, apply=False)
            opt.step(grad_scale=coef)
            return loss.detach()
        if world > 1:
            model.prepare_capture()
        graphed = GraphedStep(body, x, y, warmup=2)

        def step():                                   # noqa: F811 - the graphed replacement
            graphed(x, y)
    dt = timed_loop(step, args, comm, dev)
    sps = world * mb * args.steps / dt
    name = "ResNet-18 DDP CPU/gloo" if cpu else "ResNet-50 DDP"
    return {"metric": f"samples/sec {name} (whole node)", "value": round(sps, 2), "unit": "samples/s",
            "n_gpus": 0 if cpu else world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(1000 * dt / args.steps, 3), "higher_is_better": True, "scaling": "weak",
            **comm_fields(world), "vs_baseline": None, "dtype": "fp32" if cpu else "bf16", "data": "synthetic",
            "config": {"model": "resnet18" if cpu else "resnet50", "global_batch": world * mb, "seq_len": None,
                       "parallelism": f"dp{world}", "image": "3x224x224", "hip_graph": graph}}


def bench_swinir(args, comm, dev, world, rank):
    """The reference's own workload (Stoke-DDP.py:159,169-170,182-254): SwinIR-S x2 through the Stoke-style
    Trainer, 18 LR 128x128 -> HR 256x256 patches per device, grad_accum 2, AdamW(1e-3, (0.9, 0.99), 1e-8,
    wd 1e-4), clip-norm 0.1.  World > 1: DDP + OSS (ZeRO-1) + ShardedDDP (ZeRO-2) exactly as the reference's
    flags; world 1: no engine is needed (the bf16 compute copy still runs through the DDP flat layout).
    ``--loss feat`` is the reference's perceptual loss (Stoke-DDP.py:224; random-init feature net, parity
    unpinned), ``--loss mse`` the Fairscale script's (Fairscale-DDP.py:76).  ``--precision fp32`` is the
    reference's own precision (fp16=None, Stoke-DDP.py:247); bf16 is this framework's default.
    One step = one optimizer step (2 micro-batches)."""
    import torch
    from pytorch_distributedtraining_amd.models.losses import feat_loss
    from pytorch_distributedtraining_amd.models.swinir import swinir_s_x2
    from pytorch_distributedtraining_amd.trainer import ClipGradNormConfig, StokeOptimizer, Trainer
    mb = args.micro_batch or 18
    accum = 2
    model = swinir_s_x2()
    opt = StokeOptimizer(optimizer=torch.optim.AdamW,
                         optimizer_kwargs={"lr": 1e-3, "betas": (0.9, 0.99), "eps": 1e-8, "weight_decay": 1e-4})
    loss_fn = feat_loss if args.loss == "feat" else torch.nn.functional.mse_loss
    tr = Trainer(model, optimizer=opt, loss=loss_fn, batch_size_per_device=mb,
                 grad_accum_steps=accum, grad_clip=ClipGradNormConfig(max_norm=0.1, norm_type=2.0), gpu=dev.type == "cuda",
                 fp16=None if args.precision == "fp32" else "bf16", distributed="ddp" if world > 1 else None,
                 fairscale_oss=world > 1, fairscale_sddp=world > 1, verbose=False, comm=comm)
    g = torch.Generator(device=dev)
    g.manual_seed(2000 + rank)
    data = [(torch.rand(mb, 3, 128, 128, device=dev, generator=g), torch.rand(mb, 3, 256, 256, device=dev, generator=g))
            for _ in range(accum)]

    def step():
        for x, y in data:
            loss = tr.loss(tr.model(x), y)
            tr.backward(loss)
            tr.step()

    graph = bool(args.graph) and args.precision == "bf16" and (world == 1 or comm.backend == "nccl")
    if graph:
        # the whole optimizer step (2 micro-batches + fused AdamW) replayed as one HIP graph (Trainer.graph)
        eager_step = step
        step = tr.graph(eager_step)                    # noqa: F811
    dt = timed_loop(step, args, comm, dev)
    sps = world * mb * accum * args.steps / dt
    par = "dp{}+oss+sddp".format(world) if world > 1 else "dp1"
    return {"metric": "samples/sec SwinIR-S x2 Stoke (whole node)", "value": round(sps, 2),
            "unit": "samples/s", "n_gpus": world if dev.type == "cuda" else 0, "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000 * dt / args.steps, 3), "higher_is_better": True, "scaling": "weak",
            **comm_fields(world), "vs_baseline": None, "dtype": args.precision, "data": "synthetic",
            "config": {"model": "swinir-s-x2", "global_batch": world * mb * accum, "seq_len": None,
                       "parallelism": par, "image": "3x128x128->3x256x256", "grad_accum": accum,
                       "loss": "feat_loss (perceptual)" if args.loss == "feat" else "mse",
                       "compute_copy": tr.compute_dtype is not None, "hip_graph": graph}}


if __name__ == "__main__":
    main()
