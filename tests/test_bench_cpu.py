"""bench.py contract on CPU: ``--gpus N`` launches N ranks itself (no torchrun), rank 0 prints ONE JSON
line that reports the real world size and the engines' collective traffic; a WORLD_SIZE that disagrees
with ``--gpus`` is refused (reference launch patterns: Stoke-DDP.py:2, Fairscale-DDP.py:125-132)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(OMP_NUM_THREADS="2", **kw)
    return env


def test_bench_self_launches_two_gloo_ranks():
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--workload", "resnet18-cpu", "--steps", "1",
                        "--warmup", "1", "--micro-batch", "2"], cwd=ROOT, env=_env(), capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    res = json.loads(lines[0])
    assert res["n_ranks"] == 2
    assert res["config"]["parallelism"] == "dp2"
    assert res["config"]["global_batch"] == 4
    # DDP gradient buckets + the clip-norm scalar cross the wire every step
    assert res["collectives_per_step"] >= 2
    assert res["comm_bytes_per_step"] >= 4 * 11_000_000


def test_bench_world2_reports_topology_and_secondary_headline():
    """Both BASELINE headlines at every N (the ResNet DDP one as 'secondary'), with the c10d world size read
    back from the process group and every rank's device in 'topology'."""
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--device", "cpu", "--workload", "gpt2-fsdp",
                        "--model", "gpt2-tiny", "--micro-batch", "2", "--seq", "64", "--steps", "2", "--warmup", "1",
                        "--secondary-micro-batch", "2"], cwd=ROOT, env=_env(), capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    res = json.loads(lines[0])
    assert res["config"]["parallelism"] == "fsdp2" and res["collectives_per_step"] > 0
    topo = res["topology"]
    assert topo["c10d_world"] == 2 and topo["c10d_backend"] == "gloo"
    assert [d["rank"] for d in topo["devices"]] == [0, 1]
    sec = res["secondary"]
    assert sec["config"]["parallelism"] == "dp2" and sec["value"] > 0
    assert sec["collectives_per_step"] >= 2


def test_bench_under_torchrun_driver_command():
    """The driver's own launch form for N > 1 (torch.distributed.run, one rank per device, env:// on 127.0.0.1):
    exactly one JSON line from rank 0 with the real world size."""
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2",
                        "--device", "cpu", "--workload", "gpt2-fsdp", "--model", "gpt2-tiny", "--micro-batch", "2",
                        "--seq", "64", "--steps", "2", "--warmup", "1", "--secondary-micro-batch", "2"],
                       cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    res = json.loads(lines[0])
    assert res["n_ranks"] == 2 and res["topology"]["c10d_world"] == 2 and res["steps"] == 2
    assert res["secondary"]["config"]["parallelism"] == "dp2"


def test_bench_refuses_mismatched_world_size():
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "4", "--workload", "resnet18-cpu"], cwd=ROOT,
                       env=_env(WORLD_SIZE="2"), capture_output=True, text=True, timeout=120)
    assert r.returncode == 2
    assert "WORLD_SIZE=2" in r.stderr


def test_bench_secondary_failure_on_one_rank_keeps_primary_line():
    """a failure of the secondary ResNet measurement on ONE rank must not strand the other rank in
    a DDP collective: the ranks agree at the guarded phase boundaries, skip the secondary together, and rank 0
    still prints the primary GPT-2 line (with the reason in 'secondary_error')."""
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--device", "cpu", "--workload", "gpt2-fsdp",
                        "--model", "gpt2-tiny", "--micro-batch", "2", "--seq", "64", "--steps", "1", "--warmup", "1",
                        "--secondary-micro-batch", "2"], cwd=ROOT, env=_env(PDT_BENCH_SECONDARY_FAIL_RANK="1"),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    res = json.loads(lines[0])
    assert res["config"]["parallelism"] == "fsdp2" and res["value"] > 0
    assert "secondary" not in res
    assert "injected secondary failure" in res["secondary_error"] or "another rank" in res["secondary_error"]


def test_headline_guard_refuses_shared_gpus():
    """A GPU run at N > 1 prints a headline only when c10d world == --gpus == distinct devices."""
    import importlib.util
    import types
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    dev = types.SimpleNamespace(type="cuda")
    args = types.SimpleNamespace(gpus=4)
    good = {"metric": "m", "topology": {"c10d_world": 4, "distinct_devices": 4}}
    assert bench.headline_ok(good, args, dev, 4)
    shared = {"metric": "m", "topology": {"c10d_world": 4, "distinct_devices": 1}}
    assert not bench.headline_ok(shared, args, dev, 4)
    wrong_world = {"metric": "m", "topology": {"c10d_world": 2, "distinct_devices": 2}}
    assert not bench.headline_ok(wrong_world, args, dev, 4)
    old = os.environ.get("PDT_BENCH_REHEARSAL")
    os.environ["PDT_BENCH_REHEARSAL"] = "1"
    try:
        assert bench.headline_ok(shared, args, dev, 4) and shared["rehearsal"] and "REHEARSAL" in shared["metric"]
    finally:
        if old is None:
            del os.environ["PDT_BENCH_REHEARSAL"]
        else:
            os.environ["PDT_BENCH_REHEARSAL"] = old
    assert bench.headline_ok({"metric": "m", "topology": {}}, types.SimpleNamespace(gpus=1), dev, 1)
