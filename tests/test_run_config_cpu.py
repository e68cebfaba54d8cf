"""Run-config system: every shipped YAML loads, env overrides apply, and BASELINE.json
config 1 (ResNet-18 DDP, CPU / gloo, world_size 2) trains end to end through the launcher + Trainer
(reduced image size / steps to keep the CPU run short)."""
import glob
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_every_shipped_config_loads():
    from pytorch_distributedtraining_amd.run_config import RunConfig, load_config
    paths = sorted(glob.glob(os.path.join(ROOT, "configs", "*.yaml")))
    assert len(paths) >= 6
    models = set()
    for p in paths:
        cfg = load_config(p)
        assert isinstance(cfg, RunConfig) and cfg.batch_size_per_device > 0
        models.add(cfg.model)
    assert {"resnet18", "resnet50", "gpt2-124m", "gpt2-1.3b", "llama3-8b", "swinir-s-x2"} <= models
    sw = load_config(os.path.join(ROOT, "configs", "swinir_stoke.yaml"))
    assert (sw.grad_accum_steps, sw.grad_clip, sw.batch_size_per_device) == (2, 0.1, 18)   # Stoke-DDP.py:159,251,253
    assert sw.fairscale_oss and sw.fairscale_sddp and sw.optimizer["betas"] == (0.9, 0.99)


def test_unknown_keys_and_env_overrides(tmp_path):
    from pytorch_distributedtraining_amd.run_config import apply_env_overrides, load_config, xgmi_kwargs
    p = tmp_path / "bad.json"
    p.write_text(json.dumps({"model": "resnet18", "bogus": 1}))
    with pytest.raises(ValueError):
        load_config(str(p))
    p.write_text(json.dumps({"model": "resnet18"}))
    cfg = apply_env_overrides(load_config(str(p)), {"PDT_BUCKET_MB": "128", "PDT_FIRST_BUCKET_MB": "4",
                                                    "PDT_BATCH": "3", "PDT_STEPS": "7"})
    assert (cfg.bucket_cap_mb, cfg.first_bucket_mb, cfg.batch_size_per_device, cfg.steps) == (128.0, 4.0, 3, 7)
    assert xgmi_kwargs({"PDT_XGMI_ONESHOT_KB": "64", "PDT_XGMI_SLOT_MB": "8"}) == \
        {"oneshot_max_bytes": 65536, "slot_bytes": 8 << 20}


def test_resnet18_ddp_gloo_world2_via_launcher(tmp_path):
    cfg = tmp_path / "r18.yaml"
    src = open(os.path.join(ROOT, "configs", "resnet18_ddp_cpu.yaml")).read()
    src = src.replace("image_size: 224", "image_size: 64").replace("batch_size_per_device: 8",
                                                                   "batch_size_per_device: 2")
    src += f"\ncheckpoint_dir: {tmp_path / 'ckpt'}\nmetrics_path: {tmp_path / 'm.jsonl'}\n"
    cfg.write_text(src)
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    r = subprocess.run([sys.executable, "-m", "pytorch_distributedtraining_amd.launch", "--nproc-per-node", "2",
                        "-m", "pytorch_distributedtraining_amd.train", "--config", str(cfg)],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    final = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{") and '"world_size"' in ln]
    assert final and final[-1]["world_size"] == 2 and final[-1]["steps"] == 4
    assert final[-1]["loss"] == final[-1]["loss"]          # synced, finite
    assert glob.glob(str(tmp_path / "ckpt" / "stoke-resnet18_ddp_cpu-final-backward-step-*.pt"))
    assert os.path.getsize(tmp_path / "m.jsonl") > 0
