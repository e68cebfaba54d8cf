"""World-8 rehearsal of every engine on the CPU through torch's ``fake`` process group (tests/fake_world.py):
the engines' multi-rank code -- the nccl branches of ``Comm``, not the gloo emulation -- runs with world-8 shard
shapes and bucket plans in one process.  The same scenarios at the flagship shapes on one MI355X are in
tests/test_fake_world8_gpu.py."""
import pytest
import torch
import torch.nn as nn

from fake_world import Recorder, check_nccl_branch, fake_world

W = 8


@pytest.mark.parametrize("rank", [0, W - 1])
def test_fsdp_full_shard_world8_collectives(rank):
    from pytorch_distributedtraining_amd.models.gpt2 import build_gpt2
    from pytorch_distributedtraining_amd.optim import FusedAdamW, clip_grad_norm_
    from pytorch_distributedtraining_amd.parallel import (FullyShardedDataParallel, MixedPrecision,
                                                          ShardingStrategy)
    from pytorch_distributedtraining_amd.parallel.comm import Comm
    with fake_world(rank, W):
        torch.manual_seed(0)
        comm = Comm(xgmi=False)
        assert comm.world_size == W and comm.rank == rank and comm.backend == "fake"
        model = build_gpt2("gpt2-tiny", n_embd=64, n_head=2, n_layer=3, vocab_size=500)
        f = FullyShardedDataParallel(model, sharding_strategy=ShardingStrategy.FULL_SHARD,
                                     mixed_precision=MixedPrecision(torch.float32, torch.float32), comm=comm,
                                     device="cpu")
        units = list(f.all_units())
        for u in units:                                     # padded to a multiple of the world, 1/W each
            assert u.total % W == 0 and u.shard_numel == u.total // W
        params = f.flat_parameters()
        opt = FusedAdamW(params, lr=1e-3)
        x = torch.randint(0, 500, (2, 17))
        with Recorder() as rec:
            comm.reset_stats()
            loss = f(x[:, :-1], labels=x[:, 1:])
            loss.backward()
            clip_grad_norm_(params, 1.0, comm=comm, sharded=True)
            opt.step()
        check_nccl_branch(rec, W, max_all_reduce_numel=4)
        rs = rec.of("reduce_scatter_tensor")
        assert len(rs) == len(units)                        # one AVG reduce-scatter per unit per step
        assert all(c["op"] == "AVG" for c in rs)
        totals = sorted(u.total for u in units)
        assert sorted(int(torch.Size(c["args"][1][1]).numel()) for c in rs) == totals
        ag = rec.of("all_gather_into_tensor")
        shards = {u.shard_numel for u in units}
        assert ag and all(int(torch.Size(c["args"][1][1]).numel()) in shards for c in ag)
        # FULL_SHARD: every unit gathered for the forward, the resharded ones again for the backward
        assert len(units) <= len(ag) <= 2 * len(units)
        assert len(rec.of("all_reduce")) >= 1               # the global-norm clip: one float
        assert comm.stats["calls"] == len(rs) + len(ag) + len(rec.of("all_reduce"))


@pytest.mark.parametrize("rank", [0, W - 1])
def test_ddp_syncbn_world8_collectives(rank):
    from pytorch_distributedtraining_amd.models.resnet import resnet18
    from pytorch_distributedtraining_amd.optim import FusedAdamW
    from pytorch_distributedtraining_amd.parallel.comm import Comm
    from pytorch_distributedtraining_amd.parallel.ddp import DistributedDataParallel
    from pytorch_distributedtraining_amd.parallel.syncbn import convert_sync_batchnorm
    with fake_world(rank, W):
        torch.manual_seed(0)
        comm = Comm(xgmi=False)
        m = convert_sync_batchnorm(resnet18(num_classes=10), comm)
        n_bn = sum(1 for mod in m.modules()
                   if isinstance(mod, nn.modules.batchnorm._BatchNorm) and getattr(mod, "comm", None) is comm)
        assert n_bn == 20                                   # every BN of ResNet-18 synchronises over comm
        ddp = DistributedDataParallel(m, comm=comm, bucket_cap_mb=4.0)
        opt = FusedAdamW(ddp.optimizer_parameters(), lr=1e-3)
        x, y = torch.randn(4, 3, 32, 32), torch.randint(0, 10, (4,))
        with Recorder() as rec:
            comm.reset_stats()
            nn.functional.cross_entropy(ddp(x), y).backward()
            opt.step()
        check_nccl_branch(rec, W)
        ar = rec.of("all_reduce")
        buckets = [c for c in ar if c["op"] == "AVG"]
        stats = [c for c in ar if c["args"][0][2] == torch.float64]
        nparams = sum(p.numel() for p in m.parameters())
        # every parameter gradient crosses in exactly one AVG bucket all-reduce (bucket flats may be padded)
        assert len(buckets) == len(ddp.plan) and nparams <= sum(
            int(torch.Size(c["args"][0][1]).numel()) for c in buckets) < nparams + 64 * len(buckets)
        # SyncBN: one fp64 statistics all-reduce per layer forward and one per layer backward
        assert len(stats) == 2 * n_bn


@pytest.mark.parametrize("rank", [0, W - 1])
def test_stoke_ddp_oss_sddp_world8_collectives(rank):
    """The reference's own flags (Stoke-DDP.py:248-251): DDP + fairscale OSS + ShardedDDP, grad accumulation 2,
    clip 0.1 -- one optimizer step of a small SwinIR at world 8."""
    from pytorch_distributedtraining_amd.models.swinir import SwinIR
    from pytorch_distributedtraining_amd.parallel.comm import Comm
    from pytorch_distributedtraining_amd.trainer import ClipGradNormConfig, StokeOptimizer, Trainer
    with fake_world(rank, W):
        torch.manual_seed(0)
        comm = Comm(xgmi=False)
        model = SwinIR(img_size=16, embed_dim=12, depths=(2,), num_heads=(2,), window_size=4, upscale=2)
        opt = StokeOptimizer(optimizer=torch.optim.AdamW, optimizer_kwargs={"lr": 1e-3, "betas": (0.9, 0.99),
                                                                            "eps": 1e-8, "weight_decay": 1e-4})
        tr = Trainer(model, optimizer=opt, loss=nn.functional.mse_loss, batch_size_per_device=2,
                     grad_accum_steps=2, grad_clip=ClipGradNormConfig(max_norm=0.1, norm_type=2.0), gpu=False,
                     distributed="ddp", fairscale_oss=True, fairscale_sddp=True, verbose=False, comm=comm)
        data = [(torch.rand(2, 3, 16, 16), torch.rand(2, 3, 32, 32)) for _ in range(2)]
        with Recorder() as rec:
            comm.reset_stats()
            for x, y in data:
                tr.backward(tr.loss(tr.model(x), y))
                tr.step()
        assert tr.optimizer_steps == 1
        check_nccl_branch(rec, W)
        rs = rec.of("reduce_scatter_tensor")
        assert rs and all(c["op"] == "AVG" for c in rs)     # ZeRO-2 windows: reduced to the owners only
        assert rec.of("all_gather_into_tensor")              # OSS: updated segments back to every rank
