"""bench.py --gpus N: the launcher starts N ranks itself when torchrun did not (the driver's `python bench.py --gpus N`
form), checks WORLD_SIZE against --gpus under torchrun, and reports the process group's world size."""
import json
import os
import subprocess
import sys
from pathlib import Path
from types import SimpleNamespace

import pytest

REPO = Path(__file__).resolve().parent.parent


def _bench():
    sys.path.insert(0, str(REPO))
    import bench
    return bench


def _args(**kw):
    a = dict(gpus=None, workload="score", no_cpu_baseline=True, cpu_seconds=1.0)
    a.update(kw)
    return SimpleNamespace(**a)


def test_single_rank_runs_in_process():
    b = _bench()
    assert b.launch_command(_args(gpus=None), {}, []) is None
    assert b.launch_command(_args(gpus=1), {}, ["--gpus", "1"]) is None


def test_n_ranks_are_launched_through_torchrun():
    b = _bench()
    argv = ["--gpus", "4", "--steps", "3", "--warmup", "1"]
    cmd = b.launch_command(_args(gpus=4), {}, argv, port=29123)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29123"
    assert Path(cmd[len(cmd) - len(argv) - 1]) == REPO / "bench.py"
    assert cmd[-len(argv):] == argv  # the children get the same flags (and see WORLD_SIZE, so they do not relaunch)


def test_under_torchrun_world_size_must_match():
    b = _bench()
    assert b.launch_command(_args(gpus=2), {"WORLD_SIZE": "2"}, []) is None
    assert b.launch_command(_args(gpus=None), {"WORLD_SIZE": "8"}, []) is None
    with pytest.raises(SystemExit, match="WORLD_SIZE=2"):
        b.launch_command(_args(gpus=4), {"WORLD_SIZE": "2"}, [])


def test_parent_measures_cpu_baseline_and_hands_it_to_the_ranks(monkeypatch):
    """The parent runs the CPU baseline (no GPU in this process) and passes it to the children in the environment;
    its exit status is the children's."""
    b = _bench()
    monkeypatch.setattr(b, "cpu_baseline", lambda s: {"value": 1.5, "unit": "videos/s", "cores": 3})
    probe = [sys.executable, "-c", "import json, os, sys; d = json.loads(os.environ['VGE_BENCH_CPU_BASELINE']); "
                                   "sys.exit(0 if d['cores'] == 3 else 5)"]
    assert b.launch_ranks(_args(gpus=2, no_cpu_baseline=False), probe) == 0
    assert b.launch_ranks(_args(gpus=2, no_cpu_baseline=False),
                          [sys.executable, "-c", "import sys; sys.exit(7)"]) == 7


def test_gather_rank_times_two_gloo_ranks(tmp_path):
    """The per-rank (seconds, videos) all-gather on a world-size-2 gloo group: every rank sees both, in rank order."""
    code = (
        "import os, sys, json, torch, torch.distributed as dist\n"
        f"sys.path.insert(0, {str(REPO)!r})\n"
        "import bench\n"
        "dist.init_process_group('gloo')\n"
        "r = dist.get_rank()\n"
        "got = bench.gather_rank_times(1.0 + r, 256 + r, dist.get_world_size(), 'cpu')\n"
        f"open(os.path.join({str(tmp_path)!r}, f'r{{r}}.json'), 'w').write(json.dumps(got))\n"
        "dist.destroy_process_group()\n")
    script = tmp_path / "g.py"
    script.write_text(code)
    port = _bench()._free_port()
    subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                    "--master-addr", "127.0.0.1", "--master-port", str(port), str(script)], check=True, timeout=300)
    for r in range(2):
        assert json.loads((tmp_path / f"r{r}.json").read_text()) == [[1.0, 256], [2.0, 257]]


@pytest.mark.gpu
def test_bench_gpus_2_launches_two_ranks():
    """`python bench.py --gpus 2` (no torchrun) on the one-GPU box: two ranks (gloo, both on cuda:0) each score their
    256 clips; the line reports the process group's world size, both ranks, and value = all videos / the slowest rank."""
    env = dict(os.environ, VGE_BENCH_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
                        "--no-cpu-baseline", "--no-throughput-mode"], env=env, capture_output=True, text=True,
                       timeout=600, cwd=str(REPO))
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["ranks_seen"] == 2 and out["backend"] == "gloo"
    assert out["config"]["parallelism"] == "video-sharded x2"
    per = out["per_rank_videos_per_s"]
    assert len(per) == 2
    slowest = min(per)  # every rank scores 256 clips per step, so the slowest rank has the lowest rate
    assert out["value"] == pytest.approx(2 * slowest, rel=1e-9)
    assert out["precision"]["max_abs_ac"] < 1e-4 and out["precision"]["max_abs_tc"] < 1e-4


def test_f16_conv_kernel_choice_follows_the_library(monkeypatch):
    """bench.py names the f16 mode's conv kernel (roofline `kernel`, the PMC entry it accepts) by the rule vge_api.cpp
    applies: the staggered x3s kernel in single fp16 unless VGE_F16_X3S=0 or the stems are split (VGE_F16_MIX bit 0)."""
    bench = _bench()
    monkeypatch.delenv("VGE_F16_X3S", raising=False)
    monkeypatch.delenv("VGE_F16_MIX", raising=False)
    assert bench.f16_conv_is_x3s()
    monkeypatch.setenv("VGE_F16_MIX", "0")
    assert bench.f16_conv_is_x3s()
    monkeypatch.setenv("VGE_F16_MIX", "3")
    assert not bench.f16_conv_is_x3s()
    monkeypatch.setenv("VGE_F16_MIX", "2")
    monkeypatch.setenv("VGE_F16_X3S", "0")
    assert not bench.f16_conv_is_x3s()


def test_pmc_traffic_refuses_a_pass_of_the_other_f16_kernel(monkeypatch):
    """The committed f16 PMC pass counts for the bench line only while it was taken on the kernel the line runs."""
    bench = _bench()
    pj = json.loads((REPO / "profiles" / "pmc_conv_encoder.json").read_text())
    monkeypatch.delenv("VGE_F16_X3S", raising=False)
    monkeypatch.delenv("VGE_F16_MIX", raising=False)
    got = bench.pmc_traffic("f16", 256)
    if pj["f16"].get("source_sha") == bench._kernel_sources_sha():
        assert (got is not None) == (pj["f16"]["kernel"] == "conv_encoder_x3s_kernel")
    monkeypatch.setenv("VGE_F16_X3S", "0")
    if pj["f16"]["kernel"] == "conv_encoder_x3s_kernel":
        assert bench.pmc_traffic("f16", 256) is None


def test_nested_e2e_record_failure_is_recorded_not_raised():
    """The config-3 record of the default line runs as a child process (bench.py --workload e2e, 1 step after 1
    warm-up); when it cannot run (here: no GPU) the record says why and the config-2 line still prints."""
    if __import__("torch").cuda.is_available():
        pytest.skip("CPU-only check of the failure path")
    b = _bench()
    rec = b.run_e2e_child(SimpleNamespace(e2e_clips=2, e2e_timeout=300.0))
    assert "error" in rec and rec["error"].startswith("exit status"), rec
    assert "--workload e2e --clips 2 --steps 1 --warmup 1" in rec["cmd"]
    json.dumps(rec)
