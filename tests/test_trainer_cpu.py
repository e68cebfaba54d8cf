"""Training facade (Stoke-equivalent) on CPU: single process and gloo world_size 2, incl. the exact
option combination of the reference (ddp + OSS + ShardedDDP + grad_accum 2 + grad-norm clip +
SyncBN conversion), status validation and the checkpoint envelope round trip."""
import os

import pytest
import torch
import torch.nn as nn

from dist_utils import run_workers

from pytorch_distributedtraining_amd.trainer import (ClipGradNormConfig, DDPConfig, FairscaleOSSConfig,
                                                     StatusError, StokeOptimizer, Trainer)
from pytorch_distributedtraining_amd.utils import checkpoint as ckpt


def _model():
    torch.manual_seed(0)
    return nn.Sequential(nn.Conv2d(3, 8, 3, padding=1), nn.BatchNorm2d(8), nn.ReLU(), nn.Conv2d(8, 3, 3, padding=1))


def _opt():
    return StokeOptimizer(optimizer=torch.optim.AdamW,
                          optimizer_kwargs={"lr": 1e-3, "betas": (0.9, 0.99), "eps": 1e-8, "weight_decay": 1e-4})


def test_status_validation():
    with pytest.raises(StatusError):
        Trainer(_model(), _opt(), nn.MSELoss(), 2, fairscale_sddp=True, distributed="ddp", verbose=False)
    with pytest.raises(StatusError):
        Trainer(_model(), _opt(), nn.MSELoss(), 2, fairscale_oss=True, verbose=False)
    with pytest.raises(StatusError):
        Trainer(_model(), _opt(), nn.MSELoss(), 2, grad_accum_steps=0, verbose=False)


def test_single_process_accumulation_and_checkpoint(tmp_path):
    t = Trainer(_model(), _opt(), nn.MSELoss(), batch_size_per_device=2, grad_accum_steps=2,
                grad_clip=ClipGradNormConfig(0.1, 2.0), verbose=False)
    assert t.effective_batch_size == 4 and t.world_size == 1 and t.rank == 0
    x, y = torch.randn(2, 3, 8, 8), torch.randn(2, 3, 8, 8)
    w0 = t.model_access[0].weight.detach().clone()
    out = t.model(x)
    loss = t.loss(out, y)
    t.backward(loss)
    assert t.step() is False                                 # not a boundary yet
    assert torch.equal(w0, t.model_access[0].weight)
    t.backward(t.loss(t.model(x), y))
    assert t.step() is True
    assert not torch.equal(w0, t.model_access[0].weight)
    assert t.backward_steps == 2 and t.optimizer_steps == 1
    assert isinstance(float(t.detach_and_sync_loss(loss)), float)
    t.print_ema_loss(prepend_msg="EMA")
    path, tag = t.save(str(tmp_path), name="m1", extras={"epoch": 3})
    assert tag == "stoke-m1-backward-step-2"
    payload = torch.load(os.path.join(path, tag + ".pt"), weights_only=True)
    assert set(payload) == {"backward_step", "grad_accum_step", "optimizer_step", "stoke_status", "model_state_dict",
                            "optimizer_state_dict", "scaler_state_dict", "extras"}
    assert list(payload["model_state_dict"]) == list(_model().state_dict())    # no 'module.' prefix
    assert set(payload["optimizer_state_dict"]) == {"state", "param_groups"}
    assert ckpt.latest_checkpoint(str(tmp_path)) == tag
    t2 = Trainer(_model(), _opt(), nn.MSELoss(), batch_size_per_device=2, grad_accum_steps=2, verbose=False)
    extras = t2.load(path, tag)
    assert extras == {"epoch": 3} and t2.optimizer_steps == 1
    for a, b in zip(t.model_access.state_dict().values(), t2.model_access.state_dict().values()):
        assert torch.equal(a, b)


def test_dataloader_and_pretrained_import(tmp_path):
    from pytorch_distributedtraining_amd.data import DistributedSampler, SyntheticSRDataset, random_split
    t = Trainer(_model(), _opt(), nn.MSELoss(), batch_size_per_device=4, verbose=False)
    ds = SyntheticSRDataset(n=20, lr_size=8, scale=1)
    tr, va = random_split(ds, [0.9, 0.1], seed=1)
    assert len(tr) == 18 and len(va) == 2
    dl = t.DataLoader(tr, sampler=DistributedSampler(tr, num_replicas=1, rank=0), num_workers=0)
    xb, yb = next(iter(dl))
    assert xb.shape == (4, 3, 8, 8)
    sd = t.model_access.state_dict()
    torch.save({"params": sd}, tmp_path / "pre.pth")
    m = _model()
    ckpt.load_pretrained(m, str(tmp_path / "pre.pth"), strict=True)


def _w_trainer(rank, world, tmp):
    from pytorch_distributedtraining_amd.data import DistributedSampler, SyntheticSRDataset
    t = Trainer(_model(), _opt(), nn.MSELoss(), batch_size_per_device=2, grad_accum_steps=2,
                grad_clip=ClipGradNormConfig(0.1, 2.0), distributed="ddp", fairscale_oss=True, fairscale_sddp=True,
                configs=[DDPConfig(local_rank=rank, convert_to_sync_batch_norm=True),
                         FairscaleOSSConfig(broadcast_fp16=False)], verbose=False)
    ds = SyntheticSRDataset(n=16, lr_size=8, scale=1)
    dl = t.DataLoader(ds, sampler=DistributedSampler(ds, t.world_size, t.rank), num_workers=0)
    sched = torch.optim.lr_scheduler.OneCycleLR(t.optimizer, max_lr=0.01, pct_start=0.9, steps_per_epoch=len(dl),
                                                epochs=1)
    total = 0.0
    for x, y in dl:
        loss = t.loss(t.model(x), y)
        t.backward(loss)
        t.step()
        sched.step()
        total += t.detach_and_sync_loss(loss)
    path, tag = t.save(tmp, name="dist")
    sd = {k: v.clone() for k, v in t.model_access.state_dict().items()}
    return sd, t.optimizer_steps, type(t.model_access[1]).__name__, tag, float(total)


@pytest.mark.parametrize("world", [2, 4])
def test_distributed_trainer_reference_combination(tmp_path, world):
    """world 4 = the reference's own launch (Stoke-DDP.py:2 --nproc_per_node=4)."""
    outs = run_workers(_w_trainer, world, str(tmp_path))
    sd0, steps, bn_type, tag, _ = outs[0]
    assert steps == 8 // (2 * world) and bn_type == "SyncBatchNorm"
    for o in outs[1:]:
        for k in sd0:
            assert torch.equal(sd0[k], o[0][k]), k
    payload = torch.load(os.path.join(tmp_path, tag + ".pt"), weights_only=True)
    assert sorted(payload["optimizer_state_dict"]["state"]) == list(range(6))
    assert payload["stoke_status"]["oss"] and payload["stoke_status"]["effective_batch_size"] == 4 * world


def test_stoke_example_pretrained_flag(tmp_path):
    """examples/stoke_ddp.py --pretrained: the reference's strict pretrained import (Stoke-DDP.py:209-213)."""
    import subprocess
    import sys
    from pytorch_distributedtraining_amd.models.swinir import swinir_s_x2
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    torch.manual_seed(5)
    torch.save({"params": swinir_s_x2().state_dict()}, tmp_path / "pre.pth")
    torch.save({"params": {"bogus.weight": torch.zeros(1)}}, tmp_path / "bad.pth")
    base = [sys.executable, os.path.join(root, "examples", "stoke_ddp.py"), "--cpu", "--samples", "8", "--lr-size", "16",
            "--batchSize", "2", "--nEpochs", "1", "--ckpt-dir", str(tmp_path / "ck"), "--metrics", str(tmp_path / "m.jsonl")]
    env = dict(os.environ, OMP_NUM_THREADS="2")
    ok = subprocess.run(base + ["--pretrained", str(tmp_path / "pre.pth")], capture_output=True, text=True, env=env,
                        timeout=300)
    assert ok.returncode == 0, ok.stderr[-2000:]
    bad = subprocess.run(base + ["--pretrained", str(tmp_path / "bad.pth")], capture_output=True, text=True, env=env,
                         timeout=300)
    assert bad.returncode != 0 and "Missing key" in bad.stderr


def _w_trainer_equiv(rank, world):
    """The reference's combination (ddp + OSS + ShardedDDP + SyncBN + grad_accum 2 + clip 0.1 + OneCycle) on a
    deterministic global batch of 4: world 2 shards it 2 + 2, world 1 takes all 4."""
    torch.manual_seed(0)
    # no conv bias in front of the BatchNorm: that bias has an exactly-zero true gradient, so it would only carry
    # rounding noise that Adam amplifies into +-lr steps (no equivalence signal)
    model = nn.Sequential(nn.Conv2d(3, 8, 3, padding=1, bias=False), nn.BatchNorm2d(8), nn.ReLU(),
                          nn.Conv2d(8, 3, 3, padding=1))
    t = Trainer(model, _opt(), nn.MSELoss(), batch_size_per_device=4 // world, grad_accum_steps=2,
                grad_clip=ClipGradNormConfig(0.1, 2.0), distributed="ddp" if world > 1 else None,
                fairscale_oss=world > 1, fairscale_sddp=world > 1,
                configs=[DDPConfig(local_rank=rank, convert_to_sync_batch_norm=True),
                         FairscaleOSSConfig(broadcast_fp16=False)], verbose=False)
    sched = torch.optim.lr_scheduler.OneCycleLR(t.optimizer, max_lr=0.01, pct_start=0.9, steps_per_epoch=6, epochs=1)
    n = 4 // world
    for s in range(6):
        g = torch.Generator().manual_seed(s)
        x, y = torch.randn(4, 3, 8, 8, generator=g), torch.randn(4, 3, 8, 8, generator=g)
        t.backward(t.loss(t.model(x[rank * n:(rank + 1) * n]), y[rank * n:(rank + 1) * n]))
        t.step()
        sched.step()
    sd = t._model_state()
    return {k: v.detach().clone().float() for k, v in sd.items()}, t.optimizer_steps


@pytest.mark.parametrize("world", [2, 4])
def test_distributed_trainer_reference_combination_matches_single_process(world):
    (ref, steps1), = run_workers(_w_trainer_equiv, 1)
    outs = run_workers(_w_trainer_equiv, world)
    sd0, steps2 = outs[0]
    assert steps1 == steps2 == 3
    for k in ref:
        for o in outs[1:]:
            assert torch.equal(sd0[k], o[0][k]), k
        assert torch.allclose(sd0[k], ref[k], atol=2e-5, rtol=1e-4), (k, (sd0[k] - ref[k]).abs().max())


def _w_trainer_debug(rank, world, diverge_at):
    """PDT_COMM_DEBUG=1 PDT_VERIFY_EVERY=1: the Trainer checks the cross-rank collective sequence after every
    optimizer step.  At ``diverge_at`` the ranks issue mismatched collectives (rank 1 reduces with MAX where
    rank 0 uses SUM -- gloo runs it without complaint, the result is silently wrong)."""
    os.environ["PDT_COMM_DEBUG"] = "1"
    os.environ["PDT_VERIFY_EVERY"] = "1"
    from pytorch_distributedtraining_amd.parallel.comm import Comm
    comm = Comm()
    t = Trainer(_model(), _opt(), nn.MSELoss(), batch_size_per_device=2, grad_accum_steps=1,
                grad_clip=ClipGradNormConfig(0.1, 2.0), distributed="ddp", fairscale_oss=True, fairscale_sddp=True,
                configs=[DDPConfig(local_rank=rank)], verbose=False, comm=comm)
    g = torch.Generator().manual_seed(rank)
    for s in range(4):
        if s == diverge_at:
            x = torch.ones(1)
            t.comm.all_reduce(x, "max" if rank == 1 else "sum")
        t.backward(t.loss(t.model(torch.randn(2, 3, 8, 8, generator=g)), torch.randn(2, 3, 8, 8, generator=g)))
        try:
            t.step()
        except RuntimeError as e:
            return ("mismatch", s) if "collective mismatch" in str(e) else ("error", repr(e))
    return ("ok", None)


def test_trainer_debug_mode_catches_divergent_collective():
    assert run_workers(_w_trainer_debug, 2, -1) == [("ok", None)] * 2            # consistent run: no false alarm
    assert run_workers(_w_trainer_debug, 2, 2) == [("mismatch", 2)] * 2          # caught at that very step


def _w_lazy_loss(rank, world):
    """the facade's loss sync is lazy -- summing SyncedLoss values issues no collective and no host
    read; reading the sum issues ONE all-reduce, and equals the sum of the eagerly synced per-step means."""
    from pytorch_distributedtraining_amd.trainer import SyncedLoss, Trainer
    torch.manual_seed(0)
    t = Trainer(_model(), _opt(), nn.MSELoss(), batch_size_per_device=2, distributed="ddp", verbose=False)
    eager, lazy = 0.0, 0.0
    calls = []
    for step in range(5):
        g = torch.Generator().manual_seed(10 * step + rank)
        x, y = torch.randn(2, 3, 8, 8, generator=g), torch.randn(2, 3, 8, 8, generator=g)
        loss = t.loss(t.model(x), y)
        t.backward(loss)
        t.step()
        c0 = t.comm.stats["calls"]
        lazy = lazy + t.detach_and_sync_loss(loss, lazy=True) * 2
        calls.append(t.comm.stats["calls"] - c0)                  # no collective while summing
        d = loss.detach().reshape(1).clone()
        torch.distributed.all_reduce(d)
        eager += 2 * float(d) / world
    assert isinstance(lazy, SyncedLoss) and sum(calls) == 0
    c0 = t.comm.stats["calls"]
    v = float(lazy / 5)
    return v, eager / 5, t.comm.stats["calls"] - c0


@pytest.mark.parametrize("world", [2])
def test_lazy_synced_loss_matches_eager(world):
    outs = run_workers(_w_lazy_loss, world)
    for v, e, n in outs:
        assert abs(v - e) < 1e-5 * max(1.0, abs(e)), (v, e)
        assert n == 1                                               # one all-reduce for the whole sum
    assert outs[0][0] == outs[1][0]


def _w_ema_print(rank, world):
    """print_ema_loss (Stoke-DDP.py:76): the printed value is the EMA of the rank-averaged loss; with
    ema_print_every=3 only every third call issues a collective; detach_and_sync_loss returns Stoke's float by
    default and the lazy SyncedLoss compares / converts like a number."""
    import io
    from pytorch_distributedtraining_amd.trainer import SyncedLoss
    torch.manual_seed(0)
    t = Trainer(_model(), _opt(), nn.MSELoss(), batch_size_per_device=2, distributed="ddp", verbose=False,
                ema_print_every=3)
    out = io.StringIO()
    t.logger.stream = out
    ema, calls = None, []
    for step in range(6):
        g = torch.Generator().manual_seed(10 * step + rank)
        x, y = torch.randn(2, 3, 8, 8, generator=g), torch.randn(2, 3, 8, 8, generator=g)
        loss = t.loss(t.model(x), y)
        d = loss.detach().reshape(1).clone()
        torch.distributed.all_reduce(d)
        m = float(d) / world
        ema = m if ema is None else 0.1 * m + 0.9 * ema
        c0 = t.comm.stats["calls"]
        t.print_ema_loss(prepend_msg=f"s{step}")
        calls.append(t.comm.stats["calls"] - c0)
        t.backward(loss)
        t.step()
        if step == 3:
            expect = ema
    t.flush_prints()
    f = t.detach_and_sync_loss(loss)
    lz = t.detach_and_sync_loss(loss, lazy=True)
    ok = isinstance(f, float) and isinstance(lz, SyncedLoss) and lz == f and int(lz) == int(f) and bool(lz)
    return out.getvalue(), expect, calls, ok


def test_ema_print_every_and_loss_sync_api():
    outs = run_workers(_w_ema_print, 2)
    text0, expect, calls, ok = outs[0]
    lines = [ln for ln in text0.splitlines() if ln.startswith("s")]
    assert [ln.split(":")[0] for ln in lines] == ["s0", "s3"]            # calls 1 and 4 of 6
    assert abs(float(lines[1].split(":")[1]) - expect) < 1e-4 * max(1.0, abs(expect))
    assert outs[1][0] == ""                                             # rank 1 prints nothing
    for _, _, c, o in outs:
        assert c == [1, 0, 0, 1, 0, 0] and o                            # a collective on print calls only
