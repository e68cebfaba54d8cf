"""Engine equivalence on CPU / gloo, world_size 2: every engine must reproduce single-process training
on the concatenated global batch (DDP, ZeRO-1 OSS, ZeRO-2 ShardedDDP, FSDP full-shard / grad-op),
plus no_sync accumulation, SyncBN statistics and checkpoint consolidation."""
import copy

import pytest
import torch
import torch.nn as nn

from dist_utils import run_workers

STEPS = 3


def _model(seed=0):
    torch.manual_seed(seed)
    return nn.Sequential(nn.Linear(16, 32), nn.Tanh(), nn.Linear(32, 32), nn.Tanh(), nn.Linear(32, 4))


def _data(step, world):
    g = torch.Generator().manual_seed(100 + step)
    x = torch.randn(world * 8, 16, generator=g)
    y = torch.randn(world * 8, 4, generator=g)
    return x, y


def _reference(world, opt_cls="adamw", accum=1, clip=None):
    m = _model()
    from pytorch_distributedtraining_amd.optim import FusedAdamW, clip_grad_norm_
    opt = FusedAdamW(m.parameters(), lr=1e-2, betas=(0.9, 0.99), eps=1e-8, weight_decay=1e-4)
    for s in range(STEPS):
        for a in range(accum):
            x, y = _data(s * accum + a, world)
            loss = nn.functional.mse_loss(m(x), y) / accum
            loss.backward()
        if clip:
            clip_grad_norm_(list(m.parameters()), clip)
        opt.step()
        opt.zero_grad()
    return {k: v.detach().clone() for k, v in m.state_dict().items()}


def _shard(x, rank, world):
    n = x.shape[0] // world
    return x[rank * n:(rank + 1) * n]


def _w_ddp(rank, world, accum):
    from pytorch_distributedtraining_amd.optim import FusedAdamW
    from pytorch_distributedtraining_amd.parallel.ddp import DistributedDataParallel
    m = _model()
    ddp = DistributedDataParallel(m, bucket_cap_mb=0.001, first_bucket_mb=0.0005)
    opt = FusedAdamW(m.parameters(), lr=1e-2, betas=(0.9, 0.99), eps=1e-8, weight_decay=1e-4)
    for s in range(STEPS):
        for a in range(accum):
            x, y = _data(s * accum + a, world)
            ctx = ddp.no_sync() if a < accum - 1 else torch.enable_grad()
            with ctx:
                loss = nn.functional.mse_loss(ddp(_shard(x, rank, world)), _shard(y, rank, world)) / accum
                loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)
    return {k: v.detach().clone() for k, v in m.state_dict().items()}


@pytest.mark.parametrize("accum", [1, 2])
def test_ddp_matches_single_process(accum):
    ref = _reference(2, accum=accum)
    outs = run_workers(_w_ddp, 2, accum)
    for k in ref:
        assert torch.allclose(outs[0][k], outs[1][k], atol=0)
        assert torch.allclose(outs[0][k], ref[k], atol=2e-5), k


def _w_ddp_master(rank, world):
    """DDP compute-dtype mode (flat compute copies + fp32 master per group): only FusedAdamW.zero_grad()
    clears the accumulated flat gradient between steps."""
    from pytorch_distributedtraining_amd.optim import FusedAdamW
    from pytorch_distributedtraining_amd.parallel.ddp import DistributedDataParallel
    m = _model()
    ddp = DistributedDataParallel(m, bucket_cap_mb=0.001, first_bucket_mb=0.0005, compute_dtype=torch.float32)
    opt = FusedAdamW(ddp.optimizer_parameters(), lr=1e-2, betas=(0.9, 0.99), eps=1e-8, weight_decay=1e-4)
    for s in range(STEPS):
        x, y = _data(s, world)
        loss = nn.functional.mse_loss(ddp(_shard(x, rank, world)), _shard(y, rank, world))
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)
    return {k: v.detach().clone() for k, v in ddp.full_state_dict().items()}


def test_ddp_compute_dtype_master_matches_single_process():
    ref = _reference(2)
    outs = run_workers(_w_ddp_master, 2)
    for k in ref:
        assert torch.allclose(outs[0][k], outs[1][k], atol=0)
        assert torch.allclose(outs[0][k], ref[k], atol=2e-5), k


def _w_zero(rank, world, sddp, bcast16):
    from pytorch_distributedtraining_amd.optim import FusedAdamW
    from pytorch_distributedtraining_amd.parallel.ddp import DistributedDataParallel
    from pytorch_distributedtraining_amd.parallel.zero import OSS, ShardedDataParallel
    m = _model()
    if sddp:
        opt = OSS(m.parameters(), optim=FusedAdamW, broadcast_fp16=bcast16, lr=1e-2, betas=(0.9, 0.99), eps=1e-8,
                  weight_decay=1e-4)
        model = ShardedDataParallel(m, opt, reduce_buffer_size=256)
    else:
        model = DistributedDataParallel(m, rebuild_buckets=False)
        opt = OSS(m.parameters(), optim=FusedAdamW, broadcast_fp16=bcast16, lr=1e-2, betas=(0.9, 0.99), eps=1e-8,
                  weight_decay=1e-4)
    for s in range(STEPS):
        x, y = _data(s, world)
        model.zero_grad()
        loss = nn.functional.mse_loss(model(_shard(x, rank, world)), _shard(y, rank, world))
        loss.backward()
        opt.step()
    opt.consolidate_state_dict(0)
    sd = opt.state_dict() if rank == 0 else None
    return {k: v.detach().clone() for k, v in m.state_dict().items()}, sd, list(opt.owner)


@pytest.mark.parametrize("sddp", [False, True])
def test_zero_oss_sddp_match_single_process(sddp):
    ref = _reference(2)
    outs = run_workers(_w_zero, 2, sddp, False)
    (p0, sd, owner), (p1, _, _) = outs
    for k in ref:
        assert torch.equal(p0[k], p1[k])
        assert torch.allclose(p0[k], ref[k], atol=2e-5), k
    # consolidated optimizer state: torch layout with every parameter index
    assert sorted(sd["state"].keys()) == list(range(6))
    assert set(sd["state"][0].keys()) == {"step", "exp_avg", "exp_avg_sq"}
    assert sd["param_groups"][0]["params"] == list(range(6))
    assert set(owner) == {0, 1}


def test_oss_broadcast_fp16_close():
    ref = _reference(2)
    (p0, _, _), (p1, _, _) = run_workers(_w_zero, 2, True, True)
    # owners keep their exact fp32 shard, receivers get the fp16-compressed copy (Fairscale semantics)
    for k in ref:
        assert torch.allclose(p0[k], p1[k], atol=2e-3)
        assert torch.allclose(p0[k], ref[k], atol=5e-3), k


def _w_fsdp(rank, world, strategy):
    from pytorch_distributedtraining_amd.optim import FusedAdamW
    from pytorch_distributedtraining_amd.parallel.fsdp import (FullyShardedDataParallel, MixedPrecision,
                                                               ShardingStrategy)
    m = _model()
    f = FullyShardedDataParallel(m, wrap_classes=(nn.Linear,), sharding_strategy=ShardingStrategy(strategy),
                                 mixed_precision=MixedPrecision(torch.float32, torch.float32), device="cpu")
    opt = FusedAdamW(f.parameters(), lr=1e-2, betas=(0.9, 0.99), eps=1e-8, weight_decay=1e-4)
    for s in range(STEPS):
        x, y = _data(s, world)
        loss = nn.functional.mse_loss(f(_shard(x, rank, world)), _shard(y, rank, world))
        loss.backward()
        opt.step()
        opt.zero_grad()
    osd = f.full_optim_state_dict(opt)
    return f.state_dict(), osd


@pytest.mark.parametrize("strategy", ["full_shard", "shard_grad_op"])
def test_fsdp_matches_single_process(strategy):
    ref = _reference(2)
    (s0, o0), (s1, o1) = run_workers(_w_fsdp, 2, strategy)
    assert list(s0.keys()) == list(ref.keys())
    for k in ref:
        assert torch.equal(s0[k], s1[k])
        assert torch.allclose(s0[k], ref[k], atol=2e-5), k
    assert sorted(o0["state"].keys()) == list(range(6))
    assert o0["state"][0]["exp_avg"].shape == ref["0.weight"].shape


def _w_syncbn(rank, world):
    from pytorch_distributedtraining_amd.parallel.syncbn import convert_sync_batchnorm
    torch.manual_seed(0)
    bn = nn.BatchNorm2d(5)
    sbn = convert_sync_batchnorm(copy.deepcopy(bn))
    g = torch.Generator().manual_seed(7)
    x = torch.randn(world * 3, 5, 4, 4, generator=g)
    xs = _shard(x, rank, world).clone().requires_grad_()
    y = sbn(xs)
    (y * torch.arange(y.numel()).view_as(y).float().sin()).sum().backward()
    return y.detach(), xs.grad, sbn.running_mean.clone(), sbn.running_var.clone(), sbn.weight.grad.clone()


def test_syncbn_matches_full_batch_bn():
    outs = run_workers(_w_syncbn, 2)
    torch.manual_seed(0)
    bn = nn.BatchNorm2d(5)
    g = torch.Generator().manual_seed(7)
    x = torch.randn(6, 5, 4, 4, generator=g).requires_grad_()
    y = bn(x)
    w = torch.cat([torch.arange(y[:3].numel()).view_as(y[:3]).float().sin()] * 2)
    (y * w).sum().backward()
    for r, (yr, gr, rm, rv, gw) in enumerate(outs):
        assert torch.allclose(yr, y.detach()[r * 3:(r + 1) * 3], atol=1e-5)
        assert torch.allclose(gr, x.grad[r * 3:(r + 1) * 3], atol=1e-5)
        assert torch.allclose(rm, bn.running_mean, atol=1e-6)
        assert torch.allclose(rv, bn.running_var, atol=1e-5)
    assert torch.allclose(outs[0][4] + outs[1][4], bn.weight.grad, atol=1e-5)


def _w_sharded_save(rank, world, path):
    from pytorch_distributedtraining_amd.optim import FusedAdamW
    from pytorch_distributedtraining_amd.parallel.fsdp import FullyShardedDataParallel, MixedPrecision
    from pytorch_distributedtraining_amd.utils.sharded_checkpoint import save_sharded
    m = _model()
    f = FullyShardedDataParallel(m, wrap_classes=(nn.Linear,), mixed_precision=MixedPrecision(torch.float32,
                                 torch.float32), device="cpu")
    opt = FusedAdamW(f.parameters(), lr=1e-2)
    x, y = _data(0, world)
    nn.functional.mse_loss(f(_shard(x, rank, world)), _shard(y, rank, world)).backward()
    opt.step()
    save_sharded(path, "ck", f, opt, extras={"step": 1})
    return f.state_dict(), f.full_optim_state_dict(opt)


def _w_sharded_load(rank, world, path):
    from pytorch_distributedtraining_amd.optim import FusedAdamW
    from pytorch_distributedtraining_amd.parallel.fsdp import FullyShardedDataParallel, MixedPrecision
    from pytorch_distributedtraining_amd.utils.sharded_checkpoint import load_sharded
    m = _model(seed=123)
    f = FullyShardedDataParallel(m, wrap_classes=(nn.Linear,), mixed_precision=MixedPrecision(torch.float32,
                                 torch.float32), device="cpu")
    opt = FusedAdamW(f.parameters(), lr=1e-2)
    extras = load_sharded(path, "ck", f, opt)
    return f.state_dict(), f.full_optim_state_dict(opt), extras


def test_sharded_checkpoint_resharding(tmp_path):
    """save on 2 ranks -> load on 1 rank and on 2 ranks -> identical model + optimizer state."""
    from pytorch_distributedtraining_amd.utils.sharded_checkpoint import consolidate_to_full
    (sd, osd), _ = run_workers(_w_sharded_save, 2, str(tmp_path))
    for world in (1, 2):
        (sd2, osd2, extras) = run_workers(_w_sharded_load, world, str(tmp_path))[0]
        assert extras == {"step": 1}
        for k in sd:
            assert torch.equal(sd[k], sd2[k]), k
        for i in osd["state"]:
            assert torch.equal(osd["state"][i]["exp_avg"], osd2["state"][i]["exp_avg"])
    full, fo = consolidate_to_full(str(tmp_path), "ck")
    for k in sd:
        assert torch.equal(full[k], sd[k])
    assert torch.equal(fo["state"][0]["exp_avg_sq"], osd["state"][0]["exp_avg_sq"])


def _w_ddp_buffers(rank, world):
    from pytorch_distributedtraining_amd.parallel.ddp import DistributedDataParallel
    torch.manual_seed(0)
    m = nn.Sequential(nn.Linear(8, 8), nn.BatchNorm1d(8), nn.Linear(8, 2))
    m.register_buffer("const_table", torch.arange(1000.0))        # never written: must not be re-sent
    ddp = DistributedDataParallel(m)
    sent = []
    orig = ddp.comm.broadcast_coalesced

    def spy(tensors, *a, **k):
        sent.append(len(tensors))
        return orig(tensors, *a, **k)

    ddp.comm.broadcast_coalesced = spy
    for step in range(3):
        x = torch.randn(16, 8, generator=torch.Generator().manual_seed(100 * step + rank))
        ddp(x).sum().backward()
    bn = m[1]
    return sent, bn.running_mean.clone(), bn.num_batches_tracked.item()


def test_ddp_broadcasts_only_changed_buffers():
    """first forward syncs all 4 buffers, later ones only the 3 BatchNorm buffers; rank 1's BN
    statistics follow rank 0's each step (identical after the broadcast + identical update)."""
    (s0, rm0, n0), (s1, rm1, n1) = run_workers(_w_ddp_buffers, 2)
    assert s0 == s1 == [4, 3, 3]
    assert n0 == n1 == 3
    assert not torch.equal(rm0, rm1)   # each rank's last forward updated with its own batch
