"""The engines over the device transport, multi-rank on ONE MI355X: two ranks share cuda:0 and every
gradient / parameter collective goes through the peer-mapped xGMI kernels (parallel/xgmi.py) on each
rank's communication stream -- FSDP full-shard and shard-grad-op (all-gather + reduce-scatter), DDP with
a bf16 compute copy (bucketed all-reduce), and the reference's Stoke combination DDP + OSS + ShardedDDP
(ZeRO-2 reduce-to-owner + one all-gather of the owners' segments).  Each must match world_size 1.
Small staging slots force the chunked paths.  (RCCL refuses two ranks on one device, and gloo stages
through the host, so this is the only device transport a 1-GPU box can exercise at world 2.)
Reference combination: Stoke-DDP.py:246-252."""
import pytest
import torch
import torch.nn as nn

from dist_utils import assert_adam_close, run_workers

pytestmark = pytest.mark.gpu

SLOT = 1 << 20


def _comm(world):
    from pytorch_distributedtraining_amd.parallel import Comm
    torch.cuda.set_device(0)
    comm = Comm(xgmi=False)
    if world > 1:
        comm.enable_xgmi(slot_bytes=SLOT, oneshot_max_bytes=32 << 10)
    return comm


def _xgmi_calls(comm):
    return comm.xgmi.calls if comm.xgmi is not None else 0


def _batch(step, rank, world, dev):
    g = torch.Generator().manual_seed(step)
    x = torch.randint(0, 512, (4, 129), generator=g).to(dev)
    n = x.shape[0] // world
    return x[rank * n:(rank + 1) * n]


def _fsdp(rank, world, strategy):
    from pytorch_distributedtraining_amd.models import build_gpt2
    from pytorch_distributedtraining_amd.optim import FusedAdamW, clip_grad_norm_
    from pytorch_distributedtraining_amd.parallel import FullyShardedDataParallel
    from pytorch_distributedtraining_amd.parallel.fsdp import ShardingStrategy
    comm = _comm(world)
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    with torch.device(dev):
        m = build_gpt2("gpt2-tiny", n_embd=256, n_head=2, n_layer=2)
    f = FullyShardedDataParallel(m, comm=comm, device=dev, keep_low_precision_grads=True,
                                 sharding_strategy=ShardingStrategy(strategy))
    opt = FusedAdamW(f.flat_parameters(), lr=1e-3)
    losses = []
    for s in range(3):
        xs = _batch(s, rank, world, dev)
        loss = f(xs[:, :-1], labels=xs[:, 1:])
        loss.backward()
        _, coef, _ = clip_grad_norm_(f.flat_parameters(), 1.0, comm=comm, sharded=True, apply=False)
        opt.step(grad_scale=coef)
        opt.zero_grad()
        t = loss.detach().reshape(1).clone()
        comm.all_reduce(t, "avg")
        losses.append(float(t.item()))
    calls = _xgmi_calls(comm)
    sd = {k: v.float().cpu() for k, v in f.state_dict().items()}
    if comm.xgmi is not None:
        comm.xgmi.check()
        comm.xgmi.close()
    return losses, sd, calls


@pytest.mark.parametrize("world,strategy", [(2, "full_shard"), (2, "shard_grad_op"), (4, "full_shard")])
def test_fsdp_over_xgmi_matches_one_rank(world, strategy):
    (l1, sd1, _), = run_workers(_fsdp, 1, strategy)
    outs = run_workers(_fsdp, world, strategy)
    l2, sd2, c2 = outs[0]
    assert c2 >= 3 * 3 * 2            # per step: unit all-gathers + reduce-scatters + norm + loss on the mesh
    assert all(o[0] == l2 for o in outs)
    for a, b in zip(l1, l2):
        assert abs(a - b) < 2e-2 * abs(a)
    # the k third of the qkv bias has an exactly-zero gradient (softmax shift invariance): noise-driven Adam steps
    assert_adam_close(sd1, sd2, zero_grad_slices={"attn.c_attn.bias": slice(256, 512)})


def _ddp_bf16(rank, world):
    from pytorch_distributedtraining_amd.models import build_gpt2
    from pytorch_distributedtraining_amd.optim import FusedAdamW, clip_grad_norm_
    from pytorch_distributedtraining_amd.parallel.ddp import DistributedDataParallel
    comm = _comm(world)
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    with torch.device(dev):
        m = build_gpt2("gpt2-tiny", n_embd=256, n_head=2, n_layer=2)
    ddp = DistributedDataParallel(m, comm=comm, compute_dtype=torch.bfloat16, bucket_cap_mb=1.5, first_bucket_mb=0.25)
    params = ddp.optimizer_parameters()
    opt = FusedAdamW(params, lr=1e-3)
    for s in range(3):
        xs = _batch(s, rank, world, dev)
        ddp(xs[:, :-1], labels=xs[:, 1:]).backward()
        _, coef, _ = clip_grad_norm_(params, 1.0, comm=comm, sharded=False, apply=False)
        opt.step(grad_scale=coef)
        opt.zero_grad(set_to_none=True)
    calls = _xgmi_calls(comm)
    sd = {k: v.float().cpu() for k, v in ddp.full_state_dict().items()}
    if comm.xgmi is not None:
        comm.xgmi.check()
        comm.xgmi.close()
    return sd, calls


def test_ddp_bf16_compute_copy_over_xgmi_matches_one_rank():
    (sd1, _), = run_workers(_ddp_bf16, 1)
    (sd2, c2), (sd2b, _) = run_workers(_ddp_bf16, 2)
    assert c2 >= 3 * 2
    for k in sd1:
        assert torch.equal(sd2[k], sd2b[k]), k
        # bf16 gradients reduced in a different order (2 half-batches + a bf16 AVG vs one batch) can flip
        # the sign of near-zero components, and Adam then moves them ~lr the other way each step: the bulk
        # must agree tightly, every element within the 3-step Adam displacement
        close = torch.isclose(sd1[k], sd2[k], atol=3e-3, rtol=3e-2)
        assert close.float().mean() > 0.995, (k, float(close.float().mean()))
        assert float((sd1[k] - sd2[k]).abs().max()) <= 2 * 3 * 1e-3 + 1e-3, k


def _stoke(rank, world, sddp):
    import os
    from pytorch_distributedtraining_amd.trainer import ClipGradNormConfig, StokeOptimizer, Trainer
    os.environ["LOCAL_RANK"] = "0"          # both ranks share cuda:0 (the Trainer binds LOCAL_RANK's device)
    comm = _comm(world)
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = nn.Sequential(nn.Linear(64, 256), nn.GELU(), nn.Linear(256, 256), nn.GELU(), nn.Linear(256, 64))
    opt = StokeOptimizer(optimizer=torch.optim.AdamW,
                         optimizer_kwargs={"lr": 1e-3, "betas": (0.9, 0.99), "eps": 1e-8, "weight_decay": 1e-4})
    tr = Trainer(model, opt, nn.functional.mse_loss, batch_size_per_device=8 // world, grad_accum_steps=2,
                 grad_clip=ClipGradNormConfig(max_norm=0.5, norm_type=2.0), gpu=True, fp16="bf16",
                 distributed="ddp" if world > 1 else None, fairscale_oss=world > 1, fairscale_sddp=sddp and world > 1,
                 verbose=False, comm=comm)
    for s in range(3):
        for a in range(2):
            g = torch.Generator().manual_seed(10 * s + a)
            x = torch.randn(8, 64, generator=g).to(dev)
            y = torch.randn(8, 64, generator=g).to(dev)
            n = 8 // world
            tr.backward(tr.loss(tr.model(x[rank * n:(rank + 1) * n]), y[rank * n:(rank + 1) * n]))
            tr.step()
    calls = _xgmi_calls(comm)
    dtypes = sorted({str(p.dtype) for p in tr.model_access.parameters()})
    sd = {k: v.float().cpu() for k, v in tr._model_state().items()}
    if comm.xgmi is not None:
        comm.xgmi.check()
        comm.xgmi.close()
    return sd, calls, dtypes


@pytest.mark.parametrize("world,sddp", [(2, True), (2, False), (4, True)])
def test_stoke_ddp_oss_sddp_over_xgmi_matches_one_rank(world, sddp):
    """world 4 = the reference's own launch (Stoke-DDP.py:2)."""
    (sd1, _, dt1), = run_workers(_stoke, 1, sddp)
    outs = run_workers(_stoke, world, sddp)
    sd2, c2, dt2 = outs[0]
    assert dt1 == dt2 == ["torch.bfloat16"]      # bf16 compute copy, fp32 masters in the optimizer
    assert c2 >= 3 * 2
    for k in sd1:
        assert sd1[k].dtype == torch.float32
        for o in outs[1:]:
            assert torch.equal(sd2[k], o[0][k]), k
    assert_adam_close(sd1, sd2)
