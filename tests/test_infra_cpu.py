"""Infrastructure on CPU: models (param counts / state_dict names), checkpoint envelope helpers,
launcher failure detection + restarts, fault injection, collective consistency tracer, loaders."""
import os
import subprocess
import sys
import textwrap

import pytest
import torch

from dist_utils import run_workers

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_model_parameter_counts():
    from pytorch_distributedtraining_amd.models.gpt2 import build_gpt2
    from pytorch_distributedtraining_amd.models.llama import build_llama
    from pytorch_distributedtraining_amd.models.resnet import resnet18, resnet50
    from pytorch_distributedtraining_amd.models.swinir import swinir_s_x2
    m = swinir_s_x2()
    assert sum(p.numel() for p in m.parameters()) == 910_152           # SURVEY.md §2.D (SwinIR-S x2)
    assert len(list(m.parameters())) == 330
    assert "layers.0.residual_group.blocks.0.attn.relative_position_bias_table" in m.state_dict()
    assert abs(sum(p.numel() for p in resnet50().parameters()) - 25.557e6) < 1e4
    assert abs(sum(p.numel() for p in resnet18().parameters()) - 11.69e6) < 1e4
    with torch.device("meta"):
        assert abs(build_gpt2("gpt2-1.3b").num_params() - 1.3137e9) < 1e6
        assert abs(build_gpt2("gpt2-124m").num_params() - 124.4e6) < 1e6
        assert abs(build_llama("llama3-8b").num_params() - 8.03e9) < 1e7


def test_swinir_and_srnet_shapes():
    from pytorch_distributedtraining_amd.models.srnet import Net
    from pytorch_distributedtraining_amd.models.swinir import swinir_s_x2
    x = torch.rand(2, 3, 24, 20)
    assert swinir_s_x2()(x).shape == (2, 3, 48, 40)          # non-multiple-of-window input is padded
    assert Net(upscale_factor=2)(x).shape == (2, 3, 48, 40)


def test_llama_meta_checkpoint_conversion():
    from pytorch_distributedtraining_amd.models.llama import build_llama, convert_meta_state_dict
    m = build_llama("llama3-tiny")
    sd = m.state_dict()
    meta = {}
    h, hkv, d = 2, 1, 128
    for k, v in sd.items():
        if k.endswith("attention.wqkv.weight"):
            meta[k.replace("wqkv", "wq")] = v[: h * d]
            meta[k.replace("wqkv", "wk")] = v[h * d: (h + hkv) * d]
            meta[k.replace("wqkv", "wv")] = v[(h + hkv) * d:]
        elif k.endswith("feed_forward.w13.weight"):
            f = v.shape[0] // 2
            meta[k.replace("w13", "w1")] = v[:f]
            meta[k.replace("w13", "w3")] = v[f:]
        else:
            meta[k] = v
    back = convert_meta_state_dict(meta, m.config)
    assert set(back) == set(sd)
    for k in sd:
        assert torch.equal(back[k], sd[k])


def test_metrics_and_perceptual_loss():
    from pytorch_distributedtraining_amd.models import metrics
    from pytorch_distributedtraining_amd.models.losses import feat_loss
    a = torch.rand(2, 3, 16, 16)
    assert metrics.mae(a, a) == 0.0 and metrics.psnr(a, a) == float("inf")
    b = (a + 0.1).clamp(0, 1)
    assert 15 < metrics.psnr(a, b) < 30
    l0 = feat_loss(a, a)
    l1 = feat_loss(b, a)
    assert float(l0) == 0.0 and float(l1) > 0


def test_launcher_success_and_failure_detection(tmp_path):
    ok = tmp_path / "ok.py"
    ok.write_text("import os, sys\nsys.exit(0 if os.environ['WORLD_SIZE']=='2' else 3)\n")
    r = subprocess.run([sys.executable, "-m", "pytorch_distributedtraining_amd.launch", "--nproc-per-node", "2",
                        str(ok)], cwd=ROOT, capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    bad = tmp_path / "bad.py"
    bad.write_text(textwrap.dedent("""
        import os, sys, time
        if os.environ['RANK'] == '1':
            sys.exit(7)
        time.sleep(60)                   # the survivor must be torn down by the launcher, not hang
    """))
    counter = tmp_path / "restarts"
    r = subprocess.run([sys.executable, "-m", "pytorch_distributedtraining_amd.launch", "--nproc-per-node", "2",
                        "--max-restarts", "1", "--grace-s", "1", str(bad)], cwd=ROOT, capture_output=True, text=True,
                       timeout=60)
    assert r.returncode == 7
    assert "restarting group (1/1)" in r.stderr


def test_parse_local_rank_both_spellings(monkeypatch):
    from pytorch_distributedtraining_amd.launch import parse_local_rank
    assert parse_local_rank(["--local-rank", "3"]) == 3
    assert parse_local_rank(["--local_rank=2"]) == 2
    monkeypatch.setenv("LOCAL_RANK", "5")
    assert parse_local_rank([]) == 5
    monkeypatch.setenv("LOCAL_RANK", "None")       # the reference's failure mode (Stoke-DDP.py:153)
    assert parse_local_rank([]) == 0


def test_fault_injection_raise(monkeypatch):
    from pytorch_distributedtraining_amd.utils.fault import InjectedFault, maybe_inject_fault
    monkeypatch.setenv("PDT_FAULT_RANK", "0")
    monkeypatch.setenv("PDT_FAULT_STEP", "3")
    monkeypatch.setenv("PDT_FAULT_MODE", "raise")
    maybe_inject_fault(2)
    with pytest.raises(InjectedFault):
        maybe_inject_fault(3)


def _w_consistency(rank, world, diverge):
    from pytorch_distributedtraining_amd.parallel.comm import Comm
    c = Comm(debug=True)
    t = torch.ones(4)
    c.all_reduce(t)
    if diverge and rank == 1:
        c._trace("all_reduce:sum", torch.ones(8))     # pretend rank 1 issued a different collective
    else:
        c._trace("all_reduce:sum", torch.ones(4))
    try:
        c.verify_consistency("step 0")
        return "ok"
    except RuntimeError as e:
        return "mismatch" if "collective mismatch" in str(e) else repr(e)


def test_collective_consistency_checker():
    assert run_workers(_w_consistency, 2, False) == ["ok", "ok"]
    assert run_workers(_w_consistency, 2, True) == ["mismatch", "mismatch"]


def test_checkpoint_latest_and_atomic(tmp_path):
    from pytorch_distributedtraining_amd.utils import checkpoint as ckpt
    for step in (4, 12, 8):
        ckpt.save_checkpoint(str(tmp_path), "run", model_state={"w": torch.ones(2)}, backward_step=step)
    (tmp_path / "stoke-run-backward-step-99.pt.tmp").write_text("partial")
    assert ckpt.latest_checkpoint(str(tmp_path)) == "stoke-run-backward-step-12"
    p = ckpt.load_checkpoint(str(tmp_path), "stoke-run-backward-step-12")
    assert p["backward_step"] == 12 and torch.equal(p["model_state_dict"]["w"], torch.ones(2))


def test_device_loader_cpu_passthrough():
    from pytorch_distributedtraining_amd.data import DeviceDataLoader, SyntheticTokenDataset
    dl = DeviceDataLoader(SyntheticTokenDataset(n=10, seq_len=16, vocab=100), batch_size=4, device="cpu")
    x, y = next(iter(dl))
    assert x.shape == (4, 16) and torch.equal(x[:, 1:], y[:, :-1])
    assert len(dl) == 3


def test_window_mask_label_cache_is_identity_checked():
    """ops.window_attention caches the region labels derived from a mask buffer.  A fresh mask of the same shape
    allocated at a freed mask's address (version 0 again) must not be served the old mask's labels."""
    from pytorch_distributedtraining_amd.ops.window_attention import _mask_labels

    def swin_mask(split):
        lab = torch.zeros(2, 64, dtype=torch.long)
        lab[:, split:] = split
        return torch.where(lab[:, :, None] != lab[:, None, :], -100.0, 0.0)

    for _ in range(20):                    # the allocator hands the freed block back for the next same-size mask
        a = swin_mask(10)
        la = _mask_labels(a)
        assert la is not None and int(la[0, 63]) == 10
        ptr = a.data_ptr()
        del a
        b = swin_mask(40)
        lb = _mask_labels(b)
        assert int(lb[0, 63]) == 40 and int(lb[0, 39]) == 0, (ptr == b.data_ptr())
        del b


def test_launcher_limits_hw_queues_only_when_ranks_share_gpus(monkeypatch):
    """More ranks than GPUs (one-GPU rehearsals): <= 8 HIP hardware queues per GPU in total; one rank per GPU
    keeps the default.  The launcher counts GPUs from the env / sysfs and never through HIP (torch's
    device_count() can fall back to a HIP-initialising query) -- a HIP query here makes the test fail."""
    import torch
    from pytorch_distributedtraining_amd import launch

    def no_hip():
        raise AssertionError("the launcher must not query HIP")
    monkeypatch.setattr(torch.cuda, "device_count", no_hip)
    monkeypatch.setattr(torch._C, "_cuda_getDeviceCount", no_hip, raising=False)
    for var in ("ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(var, raising=False)
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0")
    assert launch._shared_gpu_queues(1) is None
    assert launch._shared_gpu_queues(2) == "4"
    assert launch._shared_gpu_queues(4) == "2"
    assert launch._shared_gpu_queues(8) == "1"
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,1,2,3,4,5,6,7")
    assert launch.visible_gpu_count() == 8
    assert launch._shared_gpu_queues(8) is None
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "")
    assert launch._shared_gpu_queues(4) is None
    monkeypatch.delenv("HIP_VISIBLE_DEVICES")
    n = launch.visible_gpu_count()          # sysfs KFD topology: this container has no GPU node
    assert n is None or n >= 1


def test_xgmi_size_class_routing_policy():
    """PDT_XGMI=auto routes by payload size alone (so every rank routes a collective alike): the latency class
    (<= 1 MiB by default) to the xGMI mesh, bulk to RCCL; explicit windows via PDT_XGMI_MIN_KB / _MAX_KB."""
    import pytest
    from pytorch_distributedtraining_amd.parallel.xgmi import SizeClass
    from pytorch_distributedtraining_amd.run_config import xgmi_kwargs, xgmi_mode
    assert xgmi_mode({}) == "off" and xgmi_mode({"PDT_XGMI": "0"}) == "off"
    assert xgmi_mode({"PDT_XGMI": "1"}) == "all" and xgmi_mode({"PDT_XGMI": "auto"}) == "auto"
    assert "max_bytes" not in xgmi_kwargs({"PDT_XGMI": "1"})
    kw = xgmi_kwargs({"PDT_XGMI": "auto"})
    assert kw["max_bytes"] == 1 << 20
    kw = xgmi_kwargs({"PDT_XGMI": "auto", "PDT_XGMI_MIN_KB": "4", "PDT_XGMI_MAX_KB": "256"})
    sc = SizeClass(kw["min_bytes"], kw["max_bytes"])
    assert not sc(1024) and sc(4096) and sc(256 << 10) and not sc((256 << 10) + 16)
    assert sc(4096 + 8) and SizeClass()(4)        # any size: the kernels zero-pad a partial last 16-B vector
    assert SizeClass()(16) and SizeClass()(1 << 30) and not SizeClass()(0)
    # the latency-class payloads the reference issues every step reach the mesh: the 4-byte grad-norm /
    # found_inf / loss scalars (fp32) and fp64 SyncBN statistics; gathers / scatters keep 16-byte pieces
    from types import SimpleNamespace
    from pytorch_distributedtraining_amd.parallel.xgmi import XGMIComm
    x = SimpleNamespace(size_class=SizeClass(0, 1 << 20))
    el = XGMIComm.eligible
    assert el(x, 4, "all_reduce", torch.float32) and el(x, 2 * 8 * 64, "all_reduce", torch.float64)
    assert el(x, 6, "reduce", torch.bfloat16)
    assert not el(x, 8, "all_gather", torch.float32) and not el(x, 16, "all_gather", torch.float64)
    assert not el(x, 16, "all_reduce", torch.int64) and not el(x, 2 << 20, "all_reduce", torch.float32)
    with pytest.raises(ValueError):
        SizeClass(100, 10)


def test_multi_tensor_table_layout():
    """The multi-tensor table (meta rows + packed (tensor, chunk) int32 pairs in ONE buffer, built without a
    per-chunk loop) lists every chunk of every tensor in order; empty tensors get no chunk, an empty list one dummy."""
    from pytorch_distributedtraining_amd.ops.multi_tensor import META, TensorTable
    ts = [torch.zeros(100000), torch.zeros(5), torch.zeros(0), torch.zeros(70000), torch.zeros(32768)]
    gs = [torch.zeros_like(t) for t in ts]
    tab = TensorTable([ts, gs], chunk=32768)
    want = [[i, c] for i, t in enumerate(ts) for c in range((t.numel() + 32767) // 32768)]
    assert tab.nblocks == len(want) and tab.blk.tolist() == want
    assert tab.blk.dtype == torch.int32 and tab.meta.shape == (len(ts), META)
    assert tab.meta[:, 5].tolist() == [t.numel() for t in ts]
    assert tab.meta[:, 0].tolist() == [t.data_ptr() for t in ts]
    assert tab.meta[:, 1].tolist() == [g.data_ptr() for g in gs]
    empty = TensorTable([[torch.zeros(0)]])
    assert empty.nblocks == 0 and empty.blk.tolist() == [[0, 0]]


def test_stashed_bias_grad_voided_by_in_place_write():
    """ops.attention.take_bias_grad hands back the producer's column sums only while the gradient buffer is
    unmodified since the stash (version counter shared by its views); otherwise the Linear sums dY itself."""
    from pytorch_distributedtraining_amd.ops.attention import stash_bias_grad, take_bias_grad
    g = torch.randn(4, 3, 6)
    stash_bias_grad(g, g.reshape(-1, 6).sum(0))
    assert torch.equal(take_bias_grad(g.reshape(-1, 6)), g.reshape(-1, 6).sum(0))
    assert take_bias_grad(g.reshape(-1, 6)) is None           # taken once
    stash_bias_grad(g, g.reshape(-1, 6).sum(0))
    g.reshape(-1, 6).add_(1.0)                                # e.g. a second consumer's gradient accumulated in place
    assert take_bias_grad(g.reshape(-1, 6)) is None
