"""bench.py --gpus N without an external launcher spawns its own N rank processes (CPU, gloo).

The driver's multi-GPU command may be `python3 bench.py --gpus N`; the bench must then start
the N ranks itself (as the reference's simulator starts its workers, simulation_lib/task.py:142-185)
instead of measuring one rank. --dry-run runs the multi-rank skeleton without a GPU.
"""

from __future__ import annotations

import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent


def _run(*args: str, timeout: float = 240.0) -> subprocess.CompletedProcess:
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.run([sys.executable, str(REPO / "bench.py"), *args], cwd=REPO, env=env,
                          capture_output=True, text=True, timeout=timeout)


def _json_lines(out: str) -> list[dict]:
    return [json.loads(l) for l in out.splitlines() if l.strip().startswith("{")]


@pytest.mark.parametrize("world, shards", [
    (2, [[0, 128], [128, 256]]),
    (4, [[0, 64], [64, 128], [128, 192], [192, 256]]),
])
def test_default_launch_is_one_process_driving_every_gpu(world, shards):
    # the driver's exact command, `bench.py --gpus N`: ONE child process with --procs 1 (the
    # single-process peer exchange), its line relayed
    r = _run("--gpus", str(world), "--dry-run", "--steps", "3", "--warmup", "1")
    assert r.returncode == 0, r.stderr[-3000:]
    (line,) = _json_lines(r.stdout)
    assert line["n_gpus"] == world
    assert line["config"]["workload"] == f"fedavg_resnet18_fp32_256_clients_sharded_over_{world}_gpus_one_process"
    assert line["config"]["client_shards"] == shards
    assert line["config"]["launched_by"] == "bench.py (one process)"
    assert line["config"]["launch"]["mode"] == "one process"
    assert line["config"]["exchange"]["mode"] == "peer"
    assert line["config"]["exchange"]["predicted_speedup"] > 1.0
    assert "launch_fallback" not in line["config"]
    # every N > 1 line judges the north-star speed-up itself: the same-N one-GPU anchor timed in
    # the run, measured_speedup = anchor / ms_per_step, the event-timed exchange tail
    sp = line["speedup"]
    for key in ("anchor", "measured_speedup", "aliased_ratio", "target_speedup", "meets_target", "basis", "events"):
        assert key in sp, key
    assert sp["target_speedup"] == (3.5 if world == 4 else None)
    for key in ("entry0_fold_ms", "exposed_exchange_and_finalize_ms", "predicted_exposed_exchange_and_finalize_ms"):
        assert key in sp["events"], key


def test_failed_one_process_run_falls_back_to_fresh_rank_processes():
    # an injected failure of the one-process run (as a missing peer access, a failed result
    # check or its watchdog would end it): the launcher starts N fresh rank processes whose line
    # says so
    r = _run_env({"BENCH_INJECT_FAIL": "one_process"}, "--gpus", "2", "--dry-run", "--steps", "2")
    assert r.returncode == 0, r.stderr[-3000:]
    assert "injected failure in the one_process run" in r.stderr
    assert "the single-process peer run failed (exit status 3" in r.stderr
    (line,) = _json_lines(r.stdout)
    assert line["config"]["launched_by"] == "bench.py"
    assert line["config"]["client_shards"] == [[0, 128], [128, 256]]
    assert "single-process peer run failed" in line["config"]["launch_fallback"]


def test_hung_one_process_run_is_stopped_by_its_watchdog_then_falls_back():
    import time as _time

    t0 = _time.monotonic()
    r = _run_env({"BENCH_INJECT_HANG": "0:timed:peer"}, "--gpus", "2", "--dry-run", "--steps", "2",
                 "--stage-timeout", "4")
    assert r.returncode == 0, r.stderr[-3000:]
    assert "rank 0: stage 'timed' still running after 4 s" in r.stderr
    assert "exit status 124" in r.stderr and "last stage 'timed'" in r.stderr
    (line,) = _json_lines(r.stdout)
    assert line["config"]["launched_by"] == "bench.py"
    assert _time.monotonic() - t0 < 120


def test_one_process_budget_stops_a_run_without_watchdog():
    r = _run_env({"BENCH_INJECT_HANG": "0:timed:peer"}, "--gpus", "2", "--dry-run", "--steps", "2",
                 "--stage-timeout", "0", "--one-process-timeout", "6")
    assert r.returncode == 0, r.stderr[-3000:]
    assert "still running after 6 s; the process still running, last stage 'timed'" in r.stderr
    (line,) = _json_lines(r.stdout)
    assert "single-process peer run failed" in line["config"]["launch_fallback"]


def test_no_fallback_reports_the_one_process_failure():
    r = _run_env({"BENCH_INJECT_FAIL": "one_process"}, "--gpus", "2", "--dry-run", "--no-fallback")
    assert r.returncode != 0 and _json_lines(r.stdout) == []


@pytest.mark.parametrize("world, shards", [
    (2, [[0, 128], [128, 256]]),
    (3, [[0, 85], [85, 170], [170, 256]]),
])
def test_launcher_spawns_ranks_and_relays_one_line(world, shards):
    r = _run("--gpus", str(world), "--procs", str(world), "--dry-run", "--steps", "3", "--warmup", "1")
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    line = lines[0]
    assert line["n_gpus"] == world
    assert line["config"]["workload"] == f"fedavg_resnet18_fp32_256_clients_sharded_over_{world}_gpus"
    assert line["config"]["total_clients"] == 256
    assert line["config"]["client_shards"] == shards
    assert line["config"]["launched_by"] == "bench.py"
    assert line["scaling"] == "strong" and line["steps"] == 3 and line["warmup"] == 1
    assert {"anchor", "measured_speedup", "aliased_ratio", "target_speedup", "meets_target"} <= set(line["speedup"])


def test_one_gpu_runs_in_process():
    r = _run("--gpus", "1", "--dry-run", "--steps", "2")
    assert r.returncode == 0, r.stderr[-3000:]
    (line,) = _json_lines(r.stdout)
    assert line["n_gpus"] == 1
    assert line["config"]["workload"] == "fedavg_resnet18_fp32_64_clients"
    assert line["config"]["launched_by"] == "none"


def test_failing_rank_fails_the_run():
    # every rank rejects the layout in its own argument parser: the launcher must exit non-zero
    # and relay no JSON line
    r = _run("--gpus", "2", "--dry-run", "--layout", "no_such_layout")
    assert r.returncode != 0
    assert _json_lines(r.stdout) == []
    assert "exited with status" in r.stderr


def test_launch_timeout_stops_the_ranks():
    r = _run("--gpus", "2", "--dry-run", "--launch-timeout", "0.05")
    assert r.returncode != 0
    assert _json_lines(r.stdout) == []
    assert "launch-timeout" in r.stderr


def _torchrun(extra_env: dict, *args: str) -> subprocess.CompletedProcess:
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.setdefault("OMP_NUM_THREADS", "1")
    env.update(extra_env)
    sys.path.insert(0, str(REPO))
    from bench import _free_port

    return subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
                           str(REPO / "bench.py"), "--gpus", "2", *args],
                          cwd=REPO, env=env, capture_output=True, text=True, timeout=240)


def test_external_launcher_is_respected():
    # the driver's torch.distributed.run form with --procs 2: WORLD_SIZE is set, bench.py spawns
    # nothing, every rank runs its shard
    r = _torchrun({}, "--procs", "2", "--dry-run", "--steps", "2")
    assert r.returncode == 0, r.stderr[-3000:]
    (line,) = _json_lines(r.stdout)
    assert line["n_gpus"] == 2
    assert line["config"]["launched_by"] == "external launcher"
    assert line["config"]["workload"] == "fedavg_resnet18_fp32_256_clients_sharded_over_2_gpus"


def test_external_launcher_default_is_rank_0_driving_every_gpu():
    # the default under torch.distributed.run: rank 0 runs the one-process round over every GPU of
    # the node while rank 1 waits; one line
    r = _torchrun({}, "--dry-run", "--steps", "2")
    assert r.returncode == 0, r.stderr[-3000:]
    (line,) = _json_lines(r.stdout)
    assert line["n_gpus"] == 2
    assert line["config"]["launched_by"] == "torch.distributed.run (rank 0 drives every GPU)"
    assert line["config"]["exchange"]["mode"] == "peer"


def test_external_launcher_falls_back_to_per_process_ranks_in_the_same_processes():
    r = _torchrun({"BENCH_INJECT_FAIL": "one_process"}, "--dry-run", "--steps", "2")
    assert r.returncode == 0, r.stderr[-3000:]
    (line,) = _json_lines(r.stdout)
    assert line["config"]["launched_by"] == "external launcher"
    assert line["config"]["workload"] == "fedavg_resnet18_fp32_256_clients_sharded_over_2_gpus"
    assert "single-process peer run on rank 0 failed (status 3)" in line["config"]["launch_fallback"]


def _run_env(extra_env: dict, *args: str, timeout: float = 240.0) -> subprocess.CompletedProcess:
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.setdefault("OMP_NUM_THREADS", "1")
    env.update(extra_env)
    return subprocess.run([sys.executable, str(REPO / "bench.py"), *args], cwd=REPO, env=env,
                          capture_output=True, text=True, timeout=timeout)


def test_hung_native_rank_is_named_and_the_launcher_reruns_with_torch_comm():
    # rank 1 hangs in the timed stage only with the native communicator: its watchdog ends it
    # (status 124, stage named), the launcher reports every rank's stage and starts ONE fresh set
    # of ranks with --comm torch, whose line says it is the rerun
    import time as _time

    t0 = _time.monotonic()
    r = _run_env({"BENCH_INJECT_HANG": "1:timed:native"}, "--gpus", "2", "--procs", "2", "--dry-run", "--steps", "2",
                 "--stage-timeout", "5")
    assert r.returncode == 0, r.stderr[-3000:]
    assert "rank 1: stage 'timed' still running after 5 s" in r.stderr
    assert "rank 1 exited with status 124" in r.stderr and "last stage 'timed'" in r.stderr
    assert "retrying once with fresh rank processes and --comm torch" in r.stderr
    (line,) = _json_lines(r.stdout)
    assert "--comm torch rerun" in line["config"]["launch_fallback"]
    assert _time.monotonic() - t0 < 120


def test_a_hang_in_both_runs_fails_within_the_budget():
    import time as _time

    t0 = _time.monotonic()
    r = _run_env({"BENCH_INJECT_HANG": "1:timed:any"}, "--gpus", "2", "--procs", "2", "--dry-run", "--stage-timeout", "4",
                 "--launch-timeout", "100")
    assert r.returncode != 0 and _json_lines(r.stdout) == []
    # rank 1 hangs, rank 0 waits for it in the timed stage's collective: both watchdogs fire, in the
    # run and in its one rerun
    assert r.stderr.count("rank 1: stage 'timed' still running") == 2
    assert r.stderr.count("retrying once") == 1
    assert _time.monotonic() - t0 < 100


def test_launch_timeout_names_the_stage_of_every_rank():
    # no watchdog (--stage-timeout 0): the launcher's own limit stops the run and says where each
    # rank was
    r = _run_env({"BENCH_INJECT_HANG": "0:shards:any"}, "--gpus", "2", "--procs", "2", "--dry-run", "--stage-timeout", "0",
                 "--launch-timeout", "20", "--no-fallback")
    assert r.returncode != 0
    assert "ranks still running after --launch-timeout 20 s" in r.stderr
    assert "rank 0 still running, last stage 'shards'" in r.stderr
    assert "retrying" not in r.stderr


def test_watchdog_fails_a_torchrun_job_fast():
    # the driver's launcher form: the hung rank ends itself, torchrun stops the job
    import time as _time

    t0 = _time.monotonic()
    r = _torchrun({"BENCH_INJECT_HANG": "1:timed:any"}, "--procs", "2", "--dry-run", "--stage-timeout", "5")
    assert r.returncode != 0
    # the hung rank or the one waiting for it in the stage's collective fires first; torchrun then
    # stops the other
    assert "stage 'timed' still running after 5 s" in r.stderr
    assert _time.monotonic() - t0 < 120


def test_speedup_block_labels_aliased_ratios():
    import importlib.util
    import sys as _sys

    spec = importlib.util.spec_from_file_location("bench_mod", REPO / "bench.py")
    bench = importlib.util.module_from_spec(spec)
    argv = _sys.argv
    _sys.argv = ["bench.py"]
    try:
        spec.loader.exec_module(bench)
    finally:
        _sys.argv = argv
    anchor = {"anchor_ms_per_step": 1.9}
    real = bench.speedup_block(4, 0.5, anchor, aliased=False, tail=(1.0, 0.2, 4), predicted={
        "exposed_exchange_and_finalize_ms": 0.03})
    assert real["measured_speedup"] == 3.8 and real["aliased_ratio"] is None and real["meets_target"] is True
    assert real["events"]["exposed_exchange_and_finalize_ms"] == 0.05
    assert real["events"]["predicted_exposed_exchange_and_finalize_ms"] == 0.03
    fake = bench.speedup_block(4, 1.0, anchor, aliased=True)
    assert fake["measured_speedup"] is None and fake["aliased_ratio"] == 1.9 and fake["meets_target"] is None
    assert "not a scaling figure" in fake["basis"]
