"""World-8 readiness on ONE MI355X: this process plays rank 0 or rank 7 of an 8-rank job through torch's ``fake``
process group (tests/fake_world.py) and runs one real training step of each distributed workload at its real
shapes.  Every collective takes the RCCL (nccl) branch of ``Comm`` with world-8 shard shapes; the fake group
completes it without moving data, so values are meaningless but shapes, dtypes, reduction ops, per-step counts,
bytes and this rank's peak memory are exactly those of a rank of the 8-GPU job.

  * GPT-2 1.3B FSDP FULL_SHARD, 96 x 1024 tokens per rank (BASELINE.json config 4, the flagship);
  * ResNet-50 DDP + SyncBN, 256 images per rank (config 2; Stoke-DDP.py:190-193 convert_to_sync_batch_norm);
  * SwinIR-S Stoke DDP + OSS + ShardedDDP, 18 LR 128^2 patches, grad accumulation 2, clip 0.1 (Stoke-DDP.py).
"""
import gc

import pytest
import torch
import torch.nn as nn

from fake_world import Recorder, check_nccl_branch, fake_world

pytestmark = pytest.mark.gpu
W = 8
DEV = torch.device("cuda", 0)
N1_PEAK_GB = 188.0          # the flagship's one-GPU peak (BENCH_r05 / profiles/r5)


def _fresh():
    torch.empty(1, device=DEV)          # initialise the device before touching the allocator's stats
    gc.collect()
    torch.cuda.empty_cache()
    torch.cuda.reset_peak_memory_stats(DEV)


@pytest.mark.parametrize("rank", [0, W - 1])
def test_gpt2_1p3b_fsdp_world8_step(rank):
    from pytorch_distributedtraining_amd.models.gpt2 import build_gpt2
    from pytorch_distributedtraining_amd.optim import FusedAdamW, clip_grad_norm_
    from pytorch_distributedtraining_amd.parallel import (FullyShardedDataParallel, MixedPrecision,
                                                          ShardingStrategy)
    from pytorch_distributedtraining_amd.parallel.comm import Comm
    _fresh()
    with fake_world(rank, W):
        torch.manual_seed(0)
        comm = Comm(xgmi=False)
        with torch.device(DEV):
            model = build_gpt2("gpt2-1.3b", n_positions=1024)
        mp = MixedPrecision()
        f = FullyShardedDataParallel(model, sharding_strategy=ShardingStrategy.FULL_SHARD, mixed_precision=mp,
                                     comm=comm, device=DEV, keep_low_precision_grads=True)
        units = list(f.all_units())
        params = f.flat_parameters()
        opt = FusedAdamW(params, lr=1e-4, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1)
        x = torch.randint(0, 50257, (96, 1025), device=DEV)

        def step():
            loss = f(x[:, :-1], labels=x[:, 1:])
            loss.backward()
            _, coef, _ = clip_grad_norm_(params, 1.0, comm=comm, sharded=True, apply=False)
            opt.step(grad_scale=coef)
            opt.zero_grad(set_to_none=True)
        step()                                              # first step: per-shape kernel picks
        torch.cuda.synchronize()
        torch.cuda.reset_peak_memory_stats(DEV)
        with Recorder() as rec:
            comm.reset_stats()
            step()
            torch.cuda.synchronize()
        peak = torch.cuda.max_memory_allocated(DEV) / 1e9
        check_nccl_branch(rec, W, max_all_reduce_numel=4)
        rs = rec.of("reduce_scatter_tensor")
        assert len(rs) == len(units) and all(c["op"] == "AVG" for c in rs)
        by_total = sorted(u.total for u in units)
        assert sorted(int(torch.Size(c["args"][1][1]).numel()) for c in rs) == by_total
        for c in rs:                                        # shard = padded unit total / 8, reduce dtype
            out, inp = c["args"][0], c["args"][1]
            assert int(torch.Size(out[1]).numel()) * W == int(torch.Size(inp[1]).numel())
            assert out[2] == mp.reduce_dtype and out[3] == "cuda"
        ag = rec.of("all_gather_into_tensor")
        shards = {u.shard_numel for u in units}
        assert all(int(torch.Size(c["args"][1][1]).numel()) in shards and c["args"][1][2] == mp.param_dtype
                   for c in ag)
        assert len(units) <= len(ag) <= 2 * len(units)
        nparams = sum(u.total for u in units)
        assert nparams >= 1.3137e9 and all(u.total % W == 0 for u in units)
        # bytes per step: each unit's bf16 payload gathered (fwd + the resharded bwd) and reduce-scattered once
        esz = torch.tensor([], dtype=mp.reduce_dtype).element_size()
        assert comm.stats["bytes"] >= nparams * 2 + nparams * esz
        assert peak < N1_PEAK_GB, peak                      # 1/8 of params, grads and optimizer state
        print(f"[fake world 8 rank {rank}] GPT-2 1.3B FSDP: {len(units)} units, {len(ag)} all-gathers, "
              f"{len(rs)} reduce-scatters, {comm.stats['bytes'] / 1e9:.2f} GB/step, peak {peak:.1f} GB")
    del f, model, opt
    _fresh()


@pytest.mark.parametrize("rank", [0, W - 1])
def test_resnet50_ddp_syncbn_world8_step(rank):
    from pytorch_distributedtraining_amd.models.resnet import resnet50
    from pytorch_distributedtraining_amd.optim import FusedAdamW
    from pytorch_distributedtraining_amd.parallel.comm import Comm
    from pytorch_distributedtraining_amd.parallel.ddp import DistributedDataParallel
    from pytorch_distributedtraining_amd.parallel.syncbn import convert_sync_batchnorm
    _fresh()
    with fake_world(rank, W):
        torch.manual_seed(0)
        comm = Comm(xgmi=False)
        m = convert_sync_batchnorm(resnet50().to(DEV).to(memory_format=torch.channels_last), comm)
        n_bn = sum(1 for mod in m.modules()
                   if isinstance(mod, nn.modules.batchnorm._BatchNorm) and getattr(mod, "comm", None) is comm)
        assert n_bn == 53
        ddp = DistributedDataParallel(m, comm=comm, reduce_dtype=torch.bfloat16)
        opt = FusedAdamW(ddp.optimizer_parameters(), lr=1e-3, betas=(0.9, 0.99), eps=1e-8, weight_decay=1e-4)
        x = torch.randn(256, 3, 224, 224, device=DEV).to(memory_format=torch.channels_last)
        y = torch.randint(0, 1000, (256,), device=DEV)

        def step():
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = nn.functional.cross_entropy(ddp(x), y)
            loss.backward()
            opt.step()
            opt.zero_grad(set_to_none=True)
        step()
        torch.cuda.synchronize()
        with Recorder() as rec:
            comm.reset_stats()
            step()
            torch.cuda.synchronize()
        check_nccl_branch(rec, W)
        ar = rec.of("all_reduce")
        buckets = [c for c in ar if c["op"] == "AVG"]
        stats = [c for c in ar if c["args"][0][2] == torch.float64]
        nparams = sum(p.numel() for p in m.parameters())
        assert len(buckets) == len(ddp.plan) and all(c["args"][0][2] == torch.bfloat16 for c in buckets)
        assert nparams <= sum(int(torch.Size(c["args"][0][1]).numel()) for c in buckets) < nparams + 64 * len(buckets)
        assert len(stats) == 2 * n_bn                       # SyncBN: fp64 statistics, forward and backward
        print(f"[fake world 8 rank {rank}] ResNet-50 DDP+SyncBN: {len(buckets)} bucket all-reduces, "
              f"{len(stats)} BN stat all-reduces, peak {torch.cuda.max_memory_allocated(DEV) / 1e9:.1f} GB")
    del ddp, m, opt
    _fresh()


@pytest.mark.parametrize("rank", [0, W - 1])
def test_swinir_stoke_oss_sddp_world8_step(rank):
    from pytorch_distributedtraining_amd.models.losses import feat_loss
    from pytorch_distributedtraining_amd.models.swinir import swinir_s_x2
    from pytorch_distributedtraining_amd.parallel.comm import Comm
    from pytorch_distributedtraining_amd.trainer import ClipGradNormConfig, StokeOptimizer, Trainer
    _fresh()
    with fake_world(rank, W):
        torch.manual_seed(0)
        comm = Comm(xgmi=False)
        opt = StokeOptimizer(optimizer=torch.optim.AdamW, optimizer_kwargs={"lr": 1e-3, "betas": (0.9, 0.99),
                                                                            "eps": 1e-8, "weight_decay": 1e-4})
        tr = Trainer(swinir_s_x2(), optimizer=opt, loss=feat_loss, batch_size_per_device=18, grad_accum_steps=2,
                     grad_clip=ClipGradNormConfig(max_norm=0.1, norm_type=2.0), gpu=True, fp16="bf16",
                     distributed="ddp", fairscale_oss=True, fairscale_sddp=True, verbose=False, comm=comm)
        data = [(torch.rand(18, 3, 128, 128, device=DEV), torch.rand(18, 3, 256, 256, device=DEV)) for _ in range(2)]

        def step():
            for x, y in data:
                tr.backward(tr.loss(tr.model(x), y))
                tr.step()
        step()
        torch.cuda.synchronize()
        with Recorder() as rec:
            comm.reset_stats()
            step()
            torch.cuda.synchronize()
        assert tr.optimizer_steps == 2
        check_nccl_branch(rec, W)
        rs = rec.of("reduce_scatter_tensor")
        assert rs and all(c["op"] == "AVG" for c in rs)
        ag = rec.of("all_gather_into_tensor")
        assert ag
        print(f"[fake world 8 rank {rank}] SwinIR Stoke DDP+OSS+SDDP: {len(rs)} reduce-scatters, {len(ag)} "
              f"all-gathers, {comm.stats['bytes'] / 1e6:.1f} MB/step, peak "
              f"{torch.cuda.max_memory_allocated(DEV) / 1e9:.1f} GB")
    del tr
    _fresh()
