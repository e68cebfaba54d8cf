"""Failure detection + elastic restart + auto-resume end to end on CPU / gloo: rank 1
dies at optimizer step 3, the launcher tears the group down and restarts it (``--max-restarts 1``), the
restarted ranks resume from the newest periodic checkpoint, and the run ends with exactly the parameters
of an uninterrupted run.  (The reference writes checkpoints but never reloads them, Stoke-DDP.py:137-147;
its only resilience is the W&B retry loop, :316-322.)"""
import json
import os
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _cfg(path, ckpt):
    cfg = {"name": "srnet_resume", "model": "srnet", "distributed": "ddp", "gpu": False, "backend": "gloo",
           "precision": "fp32", "batch_size_per_device": 2, "image_size": 12, "loss": "mse",
           "optimizer": {"lr": 1e-3, "betas": [0.9, 0.99], "eps": 1e-8, "weight_decay": 1e-4}, "grad_clip": 0.5,
           "steps": 6, "warmup": 0, "log_every": 100, "checkpoint_dir": ckpt, "checkpoint_every": 1}
    with open(path, "w") as f:
        json.dump(cfg, f)
    return path


def _run(tmp, tag, extra_env, restarts):
    ckpt = os.path.join(tmp, tag)
    cfg = _cfg(os.path.join(tmp, tag + ".json"), ckpt)
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(OMP_NUM_THREADS="1", **extra_env)
    r = subprocess.run([sys.executable, "-m", "pytorch_distributedtraining_amd.launch", "--nproc-per-node", "2",
                        "--max-restarts", str(restarts), "-m", "pytorch_distributedtraining_amd.train",
                        "--config", cfg], cwd=ROOT, env=env, capture_output=True, text=True, timeout=400)
    return r, ckpt


def _final(ckpt):
    files = [f for f in os.listdir(ckpt) if f.startswith("stoke-srnet_resume-final")]
    assert len(files) == 1, os.listdir(ckpt)
    return torch.load(os.path.join(ckpt, files[0]), weights_only=True)


def test_rank_failure_restart_resumes_to_identical_parameters(tmp_path):
    tmp = str(tmp_path)
    ok, ck_ok = _run(tmp, "clean", {}, 0)
    assert ok.returncode == 0, ok.stderr[-3000:]
    bad, ck_bad = _run(tmp, "fault", {"PDT_FAULT_RANK": "1", "PDT_FAULT_STEP": "3", "PDT_FAULT_MODE": "exit"}, 1)
    assert bad.returncode == 0, bad.stderr[-3000:]
    assert "rank 1 exiting at step 3" in bad.stderr
    assert "restarting group" in bad.stderr
    assert "resumed from stoke-srnet_resume-s3" in bad.stdout + bad.stderr
    a, b = _final(ck_ok), _final(ck_bad)
    assert a["optimizer_step"] == b["optimizer_step"] == 6
    for k, v in a["model_state_dict"].items():
        assert torch.equal(v, b["model_state_dict"][k]), k
    for i, st in a["optimizer_state_dict"]["state"].items():
        assert torch.equal(st["exp_avg"], b["optimizer_state_dict"]["state"][i]["exp_avg"])
