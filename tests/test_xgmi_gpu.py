"""Peer-mapped xGMI collectives (parallel/xgmi.py, csrc/kernels/xgmi_comm.hip) on ONE MI355X: 2, 4 or 8 ranks
share cuda:0 and map each other's symmetric buffers through hipIpcOpenMemHandle (the same IPC + kernel
path the 8-GPU node uses, with the peer reached over the local fabric instead of an xGMI link).
Results are checked against the exact sums computed from the ranks' deterministic inputs."""
import pytest
import torch

from dist_utils import run_workers

pytestmark = pytest.mark.gpu


def _data(rank, n, dtype, salt):
    g = torch.Generator().manual_seed(1000 * salt + rank)
    return torch.randn(n, generator=g).to(dtype)


def _xgmi_worker(rank, world):
    from pytorch_distributedtraining_amd.parallel import Comm
    torch.cuda.set_device(0)
    comm = Comm(xgmi=False)
    x = comm.enable_xgmi(slot_bytes=8 << 20, oneshot_max_bytes=64 << 10)
    out = {}
    cases = [("one_f32", 4096, torch.float32, 1), ("one_bf16", 8192, torch.bfloat16, 2),
             ("two_f32", 1 << 20, torch.float32, 3), ("two_bf16", 3 << 19, torch.bfloat16, 4)]
    for name, n, dt, salt in cases:
        for rep in range(3):        # slot alternation + epoch reuse
            t = _data(rank, n, dt, salt + 10 * rep).cuda()
            x.all_reduce(t, "sum" if rep != 1 else "avg")
            out[f"{name}_{rep}"] = t.float().cpu()
    shard = _data(rank, 5000 * 8, torch.bfloat16, 7).cuda()
    full = torch.empty(shard.numel() * world, dtype=shard.dtype, device="cuda")
    x.all_gather(full, shard)
    out["ag"] = full.float().cpu()
    inp = _data(rank, 4096 * world, torch.float32, 8).cuda()
    rs = torch.empty(4096, device="cuda")
    x.reduce_scatter(rs, inp, "avg")
    out["rs"] = rs.cpu()
    # routed through the generic Comm API (what the engines call)
    s = torch.full((4,), float(rank + 1), device="cuda")
    comm.all_reduce(s, "sum")
    out["comm_sum"] = s.cpu()
    x.barrier()
    x.check()
    x.close()
    return out


@pytest.mark.parametrize("world", [2, 4, 8])
def test_xgmi_collectives_several_ranks_on_one_gpu(world):
    """World 2 / 4 / 8 (the node size: MAXW-peer loops, two-shot chunks of 16 * world bytes, 8-way pitches)."""
    res = run_workers(_xgmi_worker, world)
    cases = [("one_f32", 4096, torch.float32, 1), ("one_bf16", 8192, torch.bfloat16, 2),
             ("two_f32", 1 << 20, torch.float32, 3), ("two_bf16", 3 << 19, torch.bfloat16, 4)]
    for name, n, dt, salt in cases:
        for rep in range(3):
            ins = [_data(r, n, dt, salt + 10 * rep).float() for r in range(world)]
            ref = sum(ins) / (world if rep == 1 else 1)
            tol = 1e-5 if dt == torch.float32 else 2e-2
            for r in range(world):
                got = res[r][f"{name}_{rep}"]
                assert torch.allclose(got, ref, atol=tol, rtol=tol), (name, rep, r, (got - ref).abs().max())
    ag_ref = torch.cat([_data(r, 5000 * 8, torch.bfloat16, 7).float() for r in range(world)])
    rs_in = [_data(r, 4096 * world, torch.float32, 8) for r in range(world)]
    for r in range(world):
        assert torch.equal(res[r]["ag"], ag_ref)
        rs_ref = sum(t[r * 4096:(r + 1) * 4096] for t in rs_in) / world
        assert torch.allclose(res[r]["rs"], rs_ref, atol=1e-6)
        assert torch.equal(res[r]["comm_sum"], torch.full((4,), float(world * (world + 1) // 2)))


def _chunked_worker(rank, world):
    from pytorch_distributedtraining_amd.parallel import Comm
    torch.cuda.set_device(0)
    comm = Comm(xgmi=False)
    x = comm.enable_xgmi(slot_bytes=1 << 20, oneshot_max_bytes=16 << 10)
    out = {}
    t = _data(rank, 3 * (1 << 18) + 40, torch.float32, 11).cuda()      # 3 MiB + 160 B: chunks + one-shot tail
    x.all_reduce(t, "sum")
    out["ar"] = t.cpu()
    shard = _data(rank, 5 * (1 << 18) // 2, torch.bfloat16, 12).cuda()  # 1.25 MiB shard, 1 MiB slot
    full = torch.empty(shard.numel() * world, dtype=shard.dtype, device="cuda")
    ev = x.all_gather(full, shard, async_op=True)
    torch.cuda.current_stream().wait_event(ev)
    out["ag"] = full.float().cpu()
    inp = _data(rank, 3 * (1 << 17) * world, torch.float32, 13).cuda()   # 1.5 MiB pieces -> 3 windows
    rs = torch.empty(3 * (1 << 17), device="cuda")
    x.reduce_scatter(rs, inp, "avg")
    out["rs"] = rs.cpu()
    r = _data(rank, (1 << 18) + 64, torch.bfloat16, 14).cuda()
    keep = r.clone()
    comm.reduce(r, dst=1, op="sum")
    out["red"] = r.float().cpu()
    out["red_keep"] = keep.float().cpu()
    x.check()
    x.close()
    return out


@pytest.mark.parametrize("world", [2, 4, 8])
def test_xgmi_chunked_collectives_and_reduce(world):
    res = run_workers(_chunked_worker, world)
    ar = sum(_data(r, 3 * (1 << 18) + 40, torch.float32, 11) for r in range(world))
    ag = torch.cat([_data(r, 5 * (1 << 18) // 2, torch.bfloat16, 12).float() for r in range(world)])
    rs_in = [_data(r, 3 * (1 << 17) * world, torch.float32, 13) for r in range(world)]
    red = sum(_data(r, (1 << 18) + 64, torch.bfloat16, 14).float() for r in range(world))
    n = 3 * (1 << 17)
    for r in range(world):
        assert torch.allclose(res[r]["ar"], ar, atol=1e-5)
        assert torch.equal(res[r]["ag"], ag)
        assert torch.allclose(res[r]["rs"], sum(t[r * n:(r + 1) * n] for t in rs_in) / world, atol=1e-6)
    assert torch.allclose(res[1]["red"], red, atol=3e-2 * world / 2, rtol=1e-2)   # the root holds the sum ...
    for r in range(world):
        if r != 1:
            assert torch.equal(res[r]["red"], res[r]["red_keep"])          # ... the others keep their input


def _timeout_worker(rank, world):
    import time
    from pytorch_distributedtraining_amd.parallel import Comm
    torch.cuda.set_device(0)
    comm = Comm(xgmi=False)
    x = comm.enable_xgmi(slot_bytes=1 << 20, timeout_us=20_000)
    if rank == 1:
        time.sleep(3.0)                      # rank 1 is late: rank 0's mesh wait runs out of budget
    t = torch.ones(4096, device="cuda")
    x.all_reduce(t, "sum")
    torch.cuda.synchronize()
    failed = x.failed()
    diag = x.diagnosis()
    raised = False
    try:
        comm.check_errors()
    except RuntimeError:
        raised = True
    nan = bool(torch.isnan(t).any())
    comm.barrier()
    x.close()
    return failed, raised, nan, diag


def test_xgmi_timeout_is_loud():
    (f0, r0, n0, d0), (f1, r1, n1, _d1) = run_workers(_timeout_worker, 2)
    assert f0 != 0 and r0 and n0             # rank 0 timed out: flag set, check raises, output poisoned
    assert f1 == 0 and not r1 and not n1     # rank 1 found rank 0's signal and completed normally
    # the diagnosis names the wait: barrier 0 of rank 0's last epoch, peer 1 still at an older epoch
    assert d0["peer"] == 1 and d0["barrier"] == 0 and d0["epoch"] == d0["issued_epoch"]
    assert d0["peer_epoch"] < d0["epoch"]


def _size_class_worker(rank, world):
    from pytorch_distributedtraining_amd.parallel import Comm
    torch.cuda.set_device(0)
    comm = Comm(xgmi=False)
    x = comm.enable_xgmi(slot_bytes=1 << 20, max_bytes=64 << 10)       # the PDT_XGMI=auto policy, 64 KiB class
    small = torch.full((1024,), float(rank + 1), device="cuda")        # 4 KiB -> mesh
    big = torch.full((1 << 18,), float(rank + 1), device="cuda")       # 1 MiB -> the c10d backend (gloo here)
    c0 = x.calls
    comm.all_reduce(small, "sum")
    c1 = x.calls
    comm.all_reduce(big, "sum")
    c2 = x.calls
    torch.cuda.synchronize()
    comm.check_errors()
    out = (c1 - c0, c2 - c1, float(small[0]), float(big[0]), float(big[-1]))
    comm.barrier()
    x.close()
    return out


def test_xgmi_size_class_routes_small_to_mesh_and_bulk_to_backend():
    exp = float(sum(r + 1 for r in range(2)))
    for mesh_small, mesh_big, s, b0, b1 in run_workers(_size_class_worker, 2):
        assert mesh_small == 1 and mesh_big == 0
        assert s == exp and b0 == exp and b1 == exp


def _trainer_latency_worker(rank, world):
    """One Stoke-facade step with the reference's per-step small collectives (Stoke-DDP.py:76,86 loss / EMA
    sync, :192 SyncBN statistics, :253 grad-norm clip with AMP's found_inf) under the PDT_XGMI=auto policy
    (1 MiB latency class): each must be carried by the mesh, not fall back to the c10d backend."""
    import torch.nn as nn
    from pytorch_distributedtraining_amd.parallel import Comm
    from pytorch_distributedtraining_amd.trainer import ClipGradNormConfig, DDPConfig, StokeOptimizer, Trainer
    torch.cuda.set_device(0)
    comm = Comm(xgmi=False)
    x = comm.enable_xgmi(slot_bytes=1 << 20, max_bytes=1 << 20)
    torch.manual_seed(0)
    model = nn.Sequential(nn.Conv2d(3, 8, 3, padding=1, bias=False), nn.BatchNorm2d(8), nn.ReLU(),
                          nn.Conv2d(8, 3, 3, padding=1))
    opt = StokeOptimizer(optimizer=torch.optim.AdamW, optimizer_kwargs={"lr": 1e-3})
    # the reference's combination (Stoke-DDP.py:246-252): DDP + OSS + ShardedDDP, so the clip norm is a sum over
    # the ranks' optimizer shards (a plain DDP replica's norm needs no collective)
    t = Trainer(model, opt, nn.MSELoss(), batch_size_per_device=2, grad_clip=ClipGradNormConfig(0.1, 2.0),
                gpu=True, fp16="amp", distributed="ddp", fairscale_oss=True, fairscale_sddp=True, comm=comm,
                configs=[DDPConfig(local_rank=rank, convert_to_sync_batch_norm=True)], verbose=False)
    g = torch.Generator().manual_seed(rank)
    xb, yb = torch.randn(2, 3, 8, 8, generator=g).cuda(), torch.randn(2, 3, 8, 8, generator=g).cuda()
    calls = {}
    c = x.calls
    out = t.model(xb)
    calls["syncbn_fwd"], c = x.calls - c, x.calls
    loss = t.loss(out, yb)
    t.backward(loss)
    calls["backward"], c = x.calls - c, x.calls
    t.step()
    calls["clip_found_inf"], c = x.calls - c, x.calls
    synced = t.detach_and_sync_loss(loss, lazy=True)
    calls["loss_lazy"], c = x.calls - c, x.calls
    v = float(synced)
    calls["loss_read"] = x.calls - c
    torch.cuda.synchronize()
    comm.check_errors()
    params = torch.cat([p.detach().float().flatten().cpu() for p in t.model_access.parameters()])
    local = float(loss.detach())
    comm.barrier()
    x.close()
    return calls, v, local, params


def test_xgmi_carries_the_per_step_latency_collectives():
    outs = run_workers(_trainer_latency_worker, 2)
    for calls, v, _, _ in outs:
        assert calls["syncbn_fwd"] >= 1, calls          # fp64 statistics (2C+1 doubles: not a 16-B multiple)
        assert calls["backward"] >= 1, calls            # SyncBN backward sums (fp64)
        assert calls["clip_found_inf"] >= 1, calls      # 4-byte norm / found_inf scalars
        assert calls["loss_lazy"] == 0 and calls["loss_read"] == 1, calls
        assert abs(v - (outs[0][2] + outs[1][2]) / 2) < 1e-5 * max(1.0, abs(v))
    assert torch.equal(outs[0][3], outs[1][3])          # replicas agree after the step
