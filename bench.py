#!/usr/bin/env python3
"""Headline benchmark: device-resident weighted FedAvg reduce on MI355X.

BASELINE.json metric: "aggregated GB/s (device-resident), N-client weighted FedAvg reduce,
1/2/4/8 GPU". One step = one full FedAvg aggregation of the resident client updates:

  N=1  (BASELINE config 2): 64 clients x ResNet-18 layout (62 tensors, 11,689,512 fp32
       params each), weights = client dataset sizes; one fused HIP launch folds the clients
       in fp64 and writes the fp32 global model; the NaN flag is read back (the reference's
       assertions) — the step ends when the host knows the round is valid.
  N>1  (BASELINE config 3): strong scaling, 256 clients in total sharded over the N ranks
       (256/N each); every rank folds its shard into an fp64 partial in tile chunks, RCCL
       exchanges each chunk while the next one is computed, and rank 0 ends with the fp32
       global model. --weak: --clients-per-gpu clients on every rank instead;
       --total-clients 256 at N=1 is the same-N single-GPU anchor.

value = algorithmic bytes of the whole job (all clients' reads + the output write) / step
time (max over ranks). Inputs are resident in HBM before the timed region. The
``roofline`` object prices the dominant kernel: algorithmic bytes per launch / its mean
duration from HIP events recorded on the launch stream inside the timed region. The
``cpu_baseline`` is the reference's CPU op sequence (oracle/ref_torch_cpu.py) on a bounded
sample of the same workload, rank 0, N=1 only.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]

Launch. ``--gpus N > 1`` without ``WORLD_SIZE`` in the environment makes this process a
launcher that never touches the GPU: it starts N fresh rank processes of this script (RANK /
LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / a free MASTER_PORT), forwards their stderr,
relays rank 0's single JSON line and exits non-zero if any rank fails or outlives
``--launch-timeout`` — the reference's simulator likewise starts its own worker processes
(simulation_lib/task.py:142-185, context.py:215-230). Under ``torch.distributed.run`` (WORLD_SIZE
set) the ranks are already there and nothing is spawned.

Failing fast (the driver gives an N > 1 run 600 s): every rank of an N > 1 run records its stage
(init, comm, tune, warmup, timed, ...) and a watchdog thread ends the rank with status 124 and the
stage's name on stderr when one stage outlives its limit (``--stage-timeout``, default 150 s; the
process group's own timeout is 120 s) — so under ``torch.distributed.run`` a hung collective ends
the job in minutes with the stuck rank named. The self-launcher (default ``--launch-timeout``
480 s) prints every rank's last stage when it stops a run, and when the ranks failed with the
library's native RCCL communicator it starts ONE fresh set of rank processes with ``--comm torch``
(the launcher never touched a GPU; no rank is re-executed); that line says so in
``config.launch_fallback``.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time
from datetime import timedelta
from pathlib import Path


def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return int(s.getsockname()[1])


def _stage_report(status_dir: str | None, n: int, running: list[int]) -> str:
    """One line per rank: its last recorded stage (BENCH_STATUS_DIR/rank<r>) and whether it runs."""
    out = []
    for r in range(n):
        stage, age = "no stage recorded", None
        if status_dir:
            try:
                p = Path(status_dir) / f"rank{r}"
                stage = p.read_text().strip() or stage
                age = time.time() - p.stat().st_mtime
            except OSError:
                pass
        state = "still running" if r in running else "exited"
        out.append(f"rank {r} {state}, last stage '{stage}'" + (f" ({age:.0f} s ago)" if age is not None else ""))
    return "; ".join(out)


def _launch_ranks(argv: list[str]) -> int | None:
    """Spawn the ranks of a ``--gpus N`` run when no launcher did (see the module docstring).

    Returns the exit code for this (parent) process, or None when this process is itself a rank
    (or a one-GPU run) and should go on to main(). Only the standard library is used here: the
    parent imports neither torch nor the package, so it never initialises the GPU and the
    children start from a clean process (no fork of a HIP runtime)."""
    import tempfile

    pre = argparse.ArgumentParser(add_help=False)
    pre.add_argument("--gpus", type=int, default=1)
    pre.add_argument("--launch-timeout", type=float, default=480.0)
    pre.add_argument("--one-process-timeout", type=float, default=200.0)
    pre.add_argument("--comm", default="native")
    pre.add_argument("--no-fallback", action="store_true")
    pre.add_argument("--procs", type=int, default=0)
    pre.add_argument("--workload", default="fedavg")
    pre.add_argument("--shard", default="clients")
    known, _ = pre.parse_known_args(argv)
    if known.gpus <= 1 or "WORLD_SIZE" in os.environ or known.procs == 1:
        return None
    deadline = time.monotonic() + known.launch_timeout
    status_dir = tempfile.mkdtemp(prefix="bench_status_")
    note = None
    if known.procs == 0 and known.workload == "fedavg" and known.shard == "clients":
        # the default: ONE process drives the N GPUs (the peer-window exchange) —
        # the reference's single server process (simulation_lib/server/server.py:122-152)
        budget = min(known.one_process_timeout, known.launch_timeout / 2)
        rc, why = _run_one_process(argv, budget, status_dir)
        if rc == 0:
            return 0
        if known.no_fallback:
            return rc
        note = f"the single-process peer run failed ({why}); this line is the per-process run"
        print(f"bench.py launcher: {note}; starting {known.gpus} fresh rank processes "
              f"({deadline - time.monotonic():.0f} s left)", file=sys.stderr)
    rank_argv = [*argv, "--procs", str(known.gpus)] if known.procs == 0 else argv
    rc, failed = _run_ranks(rank_argv, known.gpus, deadline, known.launch_timeout, status_dir, note)
    if rc != 0 and failed and known.comm == "native" and not known.no_fallback:
        left = deadline - time.monotonic()
        if left > 30.0:
            print(f"bench.py launcher: retrying once with fresh rank processes and --comm torch "
                  f"({left:.0f} s left)", file=sys.stderr)
            rerun = "native RCCL communicator run failed; this line is the --comm torch rerun"
            rc, _ = _run_ranks([*rank_argv, "--comm", "torch"], known.gpus, deadline, known.launch_timeout,
                               status_dir, f"{note}; {rerun}" if note else rerun)
    return rc


def _run_one_process(argv: list[str], budget: float, status_dir: str) -> tuple[int, str]:
    """Start ONE fresh ``bench.py --procs 1`` child for a ``--gpus N`` run and wait for it (at most
    ``budget`` s; its own stage watchdog usually ends a hang first). Relays its single JSON line
    when it exits 0; returns (exit code, why it failed). The parent touched no GPU: a failed child
    is followed by fresh per-process ranks, never by re-executing anything that initialised one."""
    import signal
    import subprocess

    env = dict(os.environ, BENCH_LAUNCHED_BY="bench.py (one process)", BENCH_STATUS_DIR=status_dir)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    try:
        (Path(status_dir) / "rank0").unlink()
    except OSError:
        pass
    p = subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__), *argv, "--procs", "1"], env=env,
                         stdout=subprocess.PIPE, stderr=None, text=True, start_new_session=True)
    try:
        out, _ = p.communicate(timeout=budget)
    except subprocess.TimeoutExpired:
        stage = _stage_report(status_dir, 1, [0])
        try:
            os.killpg(p.pid, signal.SIGKILL)
        except ProcessLookupError:
            pass
        p.communicate()
        return 1, f"still running after {budget:g} s; {stage.replace('rank 0', 'the process')}"
    lines = [ln.strip() for ln in out.splitlines() if ln.lstrip().startswith("{")]
    for ln in out.splitlines():
        if not ln.lstrip().startswith("{"):
            sys.stderr.write(ln + "\n")
    if p.returncode == 0 and len(lines) == 1:
        print(lines[0], flush=True)
        return 0, ""
    for ln in lines:  # a line that failed its result check: kept on stderr for the record
        print(f"bench.py launcher: single-process line (not relayed): {ln}", file=sys.stderr)
    if p.returncode == 0:
        return 1, f"printed {len(lines)} JSON lines (expected 1)"
    stage = _stage_report(status_dir, 1, []).replace("rank 0 exited, ", "")
    return p.returncode or 1, f"exit status {p.returncode}, {stage}"


def _run_ranks(argv: list[str], n: int, deadline: float, budget: float, status_dir: str,
               fallback_note: str | None) -> tuple[int, bool]:
    """Spawn n rank processes of this script and wait for them (see _launch_ranks). Returns (exit
    code, whether a rank failed or hung — the failures a --comm torch rerun may cure)."""
    import signal
    import subprocess
    import threading

    port = _free_port()
    procs: list[subprocess.Popen] = []
    base = dict(os.environ)
    base.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                GROUP_RANK="0", BENCH_LAUNCHED_BY="bench.py", BENCH_STATUS_DIR=status_dir)
    if fallback_note:
        base["BENCH_LAUNCH_FALLBACK"] = fallback_note
    for r in range(n):
        try:
            (Path(status_dir) / f"rank{r}").unlink()
        except OSError:
            pass
    for r in range(n):
        env = dict(base, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen(
            [sys.executable, "-u", os.path.abspath(__file__), *argv], env=env,
            stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL, stderr=None, text=True,
            start_new_session=True))  # own process group: the parent can stop a rank and its children
    json_lines: list[str] = []

    def relay() -> None:  # rank 0's stdout: the JSON line is kept, anything else goes to stderr
        assert procs[0].stdout is not None
        for line in procs[0].stdout:
            if line.lstrip().startswith("{"):
                json_lines.append(line.strip())
            else:
                sys.stderr.write(line)

    reader = threading.Thread(target=relay, daemon=True)
    reader.start()

    def stop_all() -> None:
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGTERM)
                except ProcessLookupError:
                    pass
        t_kill = time.monotonic() + 10.0
        for p in procs:
            try:
                p.wait(timeout=max(0.1, t_kill - time.monotonic()))
            except subprocess.TimeoutExpired:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
                p.wait()

    failed = None
    while True:
        codes = [p.poll() for p in procs]
        bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
        if bad:
            time.sleep(0.5)  # ranks that fail because of the first (a peer left) are reported too
            codes = [p.poll() for p in procs]
            failed = "; ".join(f"rank {r} exited with status {c}" for r, c in enumerate(codes) if c not in (None, 0))
            break
        if all(c == 0 for c in codes):
            break
        if time.monotonic() > deadline:
            failed = f"ranks still running after --launch-timeout {budget:g} s"
            break
        time.sleep(0.2)
    if failed:
        running = [r for r, p in enumerate(procs) if p.poll() is None]
        report = _stage_report(status_dir, n, running)
        stop_all()
        reader.join(timeout=5.0)
        print(f"bench.py launcher: {failed}; {report}; stopped all {n} ranks", file=sys.stderr)
        return 1, True
    reader.join(timeout=30.0)
    if len(json_lines) != 1:
        print(f"bench.py launcher: rank 0 printed {len(json_lines)} JSON lines (expected 1)", file=sys.stderr)
        return 1, False
    print(json_lines[0], flush=True)
    return 0, False


if __name__ == "__main__":
    _rc = _launch_ranks(sys.argv[1:])
    if _rc is not None:
        raise SystemExit(_rc)

import numpy as np  # noqa: E402  (after the launcher: the parent of a --gpus N run never imports torch)
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO))

from distributed_learning_simulation_lib_amd.fedavg import (  # noqa: E402
    ClientTable,
    FedAvgContext,
    ModelLayout,
    OutputTable,
    bw_probe,
)
from distributed_learning_simulation_lib_amd.sharded import (  # noqa: E402
    ExchangeModel,
    HipLocalReducer,
    RcclComm,
    chunk_edges,
    exchange_candidates,
    resolve_exchange,
    tune_exchange,
    sharded_reduce,
)

METRIC = "aggregated GB/s (device-resident), N-client weighted FedAvg reduce, 1/2/4/8 GPU"
PG_TIMEOUT_S = 120  # torch.distributed process group timeout (its collectives and rendezvous)


class _Stages:
    """A rank's current stage of an N > 1 run: written to BENCH_STATUS_DIR/rank<r> (the
    self-launcher's report when it stops a run) and watched by a daemon thread that ends the rank
    with status 124 — naming the stage on stderr — when one stage outlives its limit, so a hung
    collective cannot hold the run until the driver's kill. Test hook: BENCH_INJECT_HANG=
    "<rank>:<stage>:<comm|any>" makes that rank sleep in that stage."""

    def __init__(self) -> None:
        self.rank, self.name, self.limit = 0, "start", 0.0
        self.t = time.monotonic()
        self.comm = "native"
        self.status = None

    def start(self, rank: int, default_limit: float, comm: str) -> None:
        import threading

        self.rank, self.default, self.comm = rank, default_limit, comm
        d = os.environ.get("BENCH_STATUS_DIR")
        self.status = Path(d) / f"rank{rank}" if d else None
        if default_limit > 0 and not getattr(self, "_watching", False):
            self._watching = True  # one watchdog per process (a fallback path starts again)
            threading.Thread(target=self._watch, daemon=True).start()

    def enter(self, name: str, limit: float | None = None) -> None:
        self.name, self.t = name, time.monotonic()
        self.limit = self.default if limit is None else limit
        if self.status is not None:
            try:
                self.status.write_text(name + "\n")
            except OSError:
                pass
        hang = os.environ.get("BENCH_INJECT_HANG", "").split(":")
        if len(hang) == 3 and hang[0] == str(self.rank) and hang[1] == name and hang[2] in ("any", self.comm):
            print(f"bench.py rank {self.rank}: injected hang in stage '{name}'", file=sys.stderr, flush=True)
            while True:
                time.sleep(1.0)

    def _watch(self) -> None:
        while True:
            time.sleep(0.5)
            if self.limit > 0 and time.monotonic() - self.t > self.limit:
                print(f"bench.py rank {self.rank}: stage '{self.name}' still running after {self.limit:g} s "
                      f"(--stage-timeout); ending the rank", file=sys.stderr, flush=True)
                os._exit(124)


_STAGES = _Stages()
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


def resnet18_layout() -> ModelLayout:
    """torchvision ResNet-18 named_parameters(): 62 tensors, 11,689,512 elements."""
    shapes: list[tuple[str, tuple[int, ...]]] = [("conv1.weight", (64, 3, 7, 7)), ("bn1.weight", (64,)), ("bn1.bias", (64,))]
    cin = 64
    for li, cout in enumerate((64, 128, 256, 512), start=1):
        for b in range(2):
            pre = f"layer{li}.{b}"
            first_in = cin if b == 0 else cout
            shapes += [
                (f"{pre}.conv1.weight", (cout, first_in, 3, 3)),
                (f"{pre}.bn1.weight", (cout,)),
                (f"{pre}.bn1.bias", (cout,)),
                (f"{pre}.conv2.weight", (cout, cout, 3, 3)),
                (f"{pre}.bn2.weight", (cout,)),
                (f"{pre}.bn2.bias", (cout,)),
            ]
            if b == 0 and li > 1:
                shapes += [
                    (f"{pre}.downsample.0.weight", (cout, cin, 1, 1)),
                    (f"{pre}.downsample.1.weight", (cout,)),
                    (f"{pre}.downsample.1.bias", (cout,)),
                ]
        cin = cout
    shapes += [("fc.weight", (1000, 512)), ("fc.bias", (1000,))]
    layout = ModelLayout(names=tuple(n for n, _ in shapes), shapes=tuple(s for _, s in shapes))
    assert layout.num_segments == 62 and layout.total_numel == 11_689_512, layout.total_numel
    return layout


def vitb16_layout() -> ModelLayout:
    """torchvision ViT-B/16 named_parameters(): 152 tensors, 86,567,656 elements (config 4)."""
    d, f = 768, 3072
    shapes: list[tuple[str, tuple[int, ...]]] = [
        ("class_token", (1, 1, d)), ("conv_proj.weight", (d, 3, 16, 16)), ("conv_proj.bias", (d,)),
        ("encoder.pos_embedding", (1, 197, d)),
    ]
    for i in range(12):
        p = f"encoder.layers.encoder_layer_{i}"
        shapes += [
            (f"{p}.ln_1.weight", (d,)), (f"{p}.ln_1.bias", (d,)),
            (f"{p}.self_attention.in_proj_weight", (3 * d, d)), (f"{p}.self_attention.in_proj_bias", (3 * d,)),
            (f"{p}.self_attention.out_proj.weight", (d, d)), (f"{p}.self_attention.out_proj.bias", (d,)),
            (f"{p}.ln_2.weight", (d,)), (f"{p}.ln_2.bias", (d,)),
            (f"{p}.mlp.0.weight", (f, d)), (f"{p}.mlp.0.bias", (f,)),
            (f"{p}.mlp.3.weight", (d, f)), (f"{p}.mlp.3.bias", (d,)),
        ]
    shapes += [("encoder.ln.weight", (d,)), ("encoder.ln.bias", (d,)),
               ("heads.head.weight", (1000, d)), ("heads.head.bias", (1000,))]
    layout = ModelLayout(names=tuple(n for n, _ in shapes), shapes=tuple(s for _, s in shapes))
    assert layout.num_segments == 152 and layout.total_numel == 86_567_656, layout.total_numel
    return layout


def gpt2s_layout() -> ModelLayout:
    """GPT-2 small (HF GPT2Model) named_parameters(): 148 tensors, 124,439,808 elements (config 5)."""
    d, f = 768, 3072
    shapes: list[tuple[str, tuple[int, ...]]] = [("wte.weight", (50257, d)), ("wpe.weight", (1024, d))]
    for i in range(12):
        p = f"h.{i}"
        shapes += [
            (f"{p}.ln_1.weight", (d,)), (f"{p}.ln_1.bias", (d,)),
            (f"{p}.attn.c_attn.weight", (d, 3 * d)), (f"{p}.attn.c_attn.bias", (3 * d,)),
            (f"{p}.attn.c_proj.weight", (d, d)), (f"{p}.attn.c_proj.bias", (d,)),
            (f"{p}.ln_2.weight", (d,)), (f"{p}.ln_2.bias", (d,)),
            (f"{p}.mlp.c_fc.weight", (d, f)), (f"{p}.mlp.c_fc.bias", (f,)),
            (f"{p}.mlp.c_proj.weight", (f, d)), (f"{p}.mlp.c_proj.bias", (d,)),
        ]
    shapes += [("ln_f.weight", (d,)), ("ln_f.bias", (d,))]
    layout = ModelLayout(names=tuple(n for n, _ in shapes), shapes=tuple(s for _, s in shapes))
    assert layout.num_segments == 148 and layout.total_numel == 124_439_808, layout.total_numel
    return layout


LAYOUTS = {
    "resnet18": resnet18_layout,
    "vitb16": vitb16_layout,
    "gpt2s": gpt2s_layout,
    "flat1m": lambda: ModelLayout.flat(1_000_000),
}


def dataset_size_weights(n: int, seed: int = 99) -> list[int]:
    rng = np.random.default_rng(seed)
    return [int(x) for x in rng.integers(100, 5001, size=n)]


def make_clients(layout: ModelLayout, first_client: int, n: int, device: torch.device, dtype: torch.dtype):
    """n synthetic client buckets x ~ N(0,1), seeded per global client id, resident in HBM."""
    offs, padded = layout.padded_offsets(torch.empty((), dtype=dtype).element_size())
    buckets = torch.empty((n, padded), dtype=dtype, device=device)
    g = torch.Generator(device=device)
    for i in range(n):
        g.manual_seed(1234 + first_client + i)
        buckets[i].normal_(generator=g)
    views = [[buckets[i, o : o + m] for o, m in zip(offs, layout.numels)] for i in range(n)]
    return buckets, views


def sample_elements(layout: ModelLayout, k_random: int = 4096, seed: int = 7) -> list[tuple[int, int]]:
    """The (segment, index-in-segment) pairs a result check reads: every tensor's first and last
    element plus ``k_random`` elements drawn uniformly over the model (seeded), in model order."""
    rng = np.random.default_rng(seed)
    starts = np.cumsum([0] + layout.numels[:-1])
    picks = set()
    for s, m in enumerate(layout.numels):
        picks.update({(s, 0), (s, m - 1)})
    for e in rng.integers(0, layout.total_numel, size=k_random):
        s = int(np.searchsorted(starts, e, side="right") - 1)
        picks.add((s, int(e - starts[s])))
    return sorted(picks)


def flat_index(layout: ModelLayout, picks: list[tuple[int, int]], elem_bytes: int, device: torch.device) -> torch.Tensor:
    """Positions of ``picks`` in a padded flat buffer of the layout (ModelLayout.padded_offsets)."""
    offs, _ = layout.padded_offsets(elem_bytes)
    return torch.tensor([offs[s] + i for s, i in picks], dtype=torch.int64, device=device)


def gather_client_samples(buckets: torch.Tensor, idx: torch.Tensor, first_client: int) -> tuple[np.ndarray, int]:
    """The sampled elements of every resident client row ([n, K] fp64, exact) and how many rows
    differ from their regeneration from the client's seed (make_clients): 0 = the inputs the
    timed rounds read are intact — no stray store (a peer store that missed its slot) touched them."""
    samples = buckets[:, idx].to(torch.float64).cpu().numpy()
    g = torch.Generator(device=buckets.device)
    scratch = torch.empty((1, buckets.shape[1]), dtype=buckets.dtype, device=buckets.device)
    changed = 0
    for i in range(buckets.shape[0]):
        g.manual_seed(1234 + first_client + i)
        scratch[0].normal_(generator=g)
        changed += int(not torch.equal(scratch[0], buckets[i]))
    del scratch
    return samples, changed


def _ordered_bits(a: np.ndarray) -> np.ndarray:
    """IEEE bits mapped to a monotone integer line (+0 and -0 both at 0): ulp distance = difference."""
    if a.dtype == np.float32:
        i = a.view(np.int32).astype(np.int64)
        return np.where(i < 0, -(i & 0x7FFFFFFF), i)
    i = a.astype(np.float64).view(np.int64)
    return np.where(i < 0, -(i & 0x7FFFFFFFFFFFFFFF), i)


def result_check(got: np.ndarray, shards: list[np.ndarray], shard_weights: list[list[float]], out_dtype: str,
                 exact: str | None) -> dict:
    """Check sampled result elements against host fp64 compositions of the same clients
    (fed_avg_algorithm.py:43-99: ``tmp = x.to(f64) * w; acc += tmp`` in arrival order, ``acc / W``).

    ``shards[g]``: [n_g, K] fp64 client samples of entry / rank g in arrival order. ``exact``:
    "single" — the one-GPU kernel, bit-identical to the reference's single chain; "composition" —
    the peer exchange, bit-identical to each shard's chain summed in shard order; None — RCCL's
    summation order, within the stated tolerance of the single chain (|Δ| ≤ 1e-12 · Σ|w x| / W in
    fp64, ≤ 1 ulp after an fp32 cast — or |Δ| within that fp64 bound plus half an ulp of the output
    where the result nearly cancels). Every form is also compared with the single chain."""
    K = got.shape[0]
    W = -0.0
    for ws in shard_weights:
        for w in ws:
            W += w
    parts, single, mag = [], np.full(K, -0.0), np.zeros(K)
    for xs, ws in zip(shards, shard_weights):
        acc = np.full(K, -0.0)
        for x, w in zip(xs, ws):
            acc = acc + x * w
            single = single + x * w
            mag = mag + np.abs(x * w)
        if len(ws):
            parts.append(acc)
    comp = parts[0]
    for p in parts[1:]:
        comp = comp + p
    npdt = np.float32 if out_dtype == "float32" else np.float64
    want_single = (single / W).astype(npdt)
    want_comp = (comp / W).astype(npdt)
    got = got.astype(npdt)
    bound = 1e-12 * mag / abs(W)
    diff = np.abs(got.astype(np.float64) - single / W)
    ulp = np.abs(_ordered_bits(got) - _ordered_bits(want_single))
    if npdt == np.float64:
        within = diff <= bound
    else:
        half_ulp = np.spacing(np.abs(want_single)).astype(np.float64) / 2
        within = (ulp <= 1) | (diff <= bound + half_ulp)
    bits_single = bool(np.array_equal(_ordered_bits(got), _ordered_bits(want_single)))
    bits_comp = bool(np.array_equal(_ordered_bits(got), _ordered_bits(want_comp)))
    ok = bool(np.all(within)) and (exact is None or (bits_single if exact == "single" else bits_comp))
    return {
        "elements": int(K), "expected": exact or "tolerance",
        "bit_identical_to_single_chain": bits_single, "bit_identical_to_shard_composition": bits_comp,
        "max_abs_vs_single_chain": float(np.abs(got.astype(np.float64) - want_single.astype(np.float64)).max()),
        "max_ulp_vs_single_chain": int(ulp.max()), "within_tolerance": bool(np.all(within)), "ok": ok,
    }


def hbm_probes(device: torch.device, nbytes: int = 4 << 30) -> dict:
    src = torch.empty(nbytes // 4, dtype=torch.float32, device=device).fill_(1.0)
    dst = torch.empty_like(src)
    out = {}
    for mode, name, moved in ((0, "copy", 2 * nbytes), (1, "read", nbytes)):
        for _ in range(2):
            bw_probe(src, dst, mode)
        torch.cuda.synchronize(device)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 10
        e0.record()
        for _ in range(reps):
            bw_probe(src, dst, mode)
        e1.record()
        torch.cuda.synchronize(device)
        ms = e0.elapsed_time(e1) / reps
        out[f"{name}_GBps"] = round(moved / (ms * 1e-3) / 1e9, 1)
    del src, dst
    torch.cuda.empty_cache()
    return out


def host_cpu() -> dict:
    """The host the CPU baseline ran on (its rate moves several-fold between the pool's boxes: the
    model, the CPUs this process may use, and the machine's total)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        usable = None
    out = {"model": model, "usable_cpus": usable, "machine_cpus": os.cpu_count(),
           "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and usable and int(omp) < usable:
        # the GPU pool runs one GPU's job per box share: OMP_NUM_THREADS is set to that share
        # (16 CPUs per GPU) by the harness, while the affinity mask shows the whole machine
        out["cores_note"] = (f"timed on OMP_NUM_THREADS={omp} threads: the harness's per-GPU CPU share on this "
                             f"box (its affinity mask shows all {usable} CPUs of the machine, shared by 8 GPUs' jobs)")
    return out


def gpu_local_cpus(device_index: int = 0) -> tuple[list[int], str]:
    """CPUs on the GPU's own NUMA node (sysfs ``local_cpulist`` of its PCI function), among those this
    process may use — where a CPU baseline beside this GPU's job should run — and where they came from."""
    usable = sorted(os.sched_getaffinity(0))
    try:
        pr = torch.cuda.get_device_properties(device_index)
        bdf = f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}.0"
        text = Path(f"/sys/bus/pci/devices/{bdf}/local_cpulist").read_text().strip()
    except (AttributeError, OSError, RuntimeError, AssertionError):
        return usable, "affinity mask (the GPU's NUMA node is not readable here)"
    local: set[int] = set()
    for part in text.split(","):
        lo, _, hi = part.partition("-")
        local.update(range(int(lo), int(hi or lo) + 1))
    mine = [c for c in usable if c in local]
    return (mine, f"local_cpulist of the GPU's PCI function {bdf}") if mine else (usable, "affinity mask")


def _cpu_baseline_child(spec: dict) -> dict:
    """Runs in a fresh process (bench.py --cpu-baseline-child): pinned to the chosen CPUs before torch
    starts its thread pool, then the reference's round timed ``repeats`` times."""
    os.sched_setaffinity(0, spec["cpus"])
    torch.set_num_threads(spec["threads"])
    sys.path.insert(0, str(REPO))
    from distributed_learning_simulation_lib_amd.message import ParameterMessage
    from oracle.ref_torch_cpu import RefFedAvgAlgorithm

    layout = LAYOUTS[spec["layout"]]()
    dtype = getattr(torch, spec["dtype"])
    n_clients = spec["clients"]
    weights = dataset_size_weights(n_clients)
    clients = []
    for i in range(n_clients):  # generation is outside the timed region
        g = torch.Generator().manual_seed(1234 + i)
        clients.append({n: torch.randn(s, generator=g, dtype=torch.float32).to(dtype)
                        for n, s in zip(layout.names, layout.shapes)})
    times = []
    t_start = time.perf_counter()
    load0 = os.getloadavg()
    while len(times) < spec["repeats"] and (len(times) < 3 or time.perf_counter() - t_start < spec["budget_s"]):
        msgs = [ParameterMessage(parameter=dict(c), aggregation_weight=w) for c, w in zip(clients, weights)]
        algo = RefFedAvgAlgorithm()
        t0 = time.perf_counter()
        for wid, m in enumerate(msgs):
            algo.process_worker_data(wid, m)
        out = algo.aggregate_worker_data()
        times.append(time.perf_counter() - t0)
        del out, algo, msgs
    return {"times_s": times, "wall_s": time.perf_counter() - t_start, "loadavg_before": load0,
            "loadavg_after": os.getloadavg(), "threads_seen": torch.get_num_threads()}


def cpu_baseline(layout: ModelLayout, n_clients: int = 64, repeats: int = 5, dtype: torch.dtype = torch.float32,
                 budget_s: float = 20.0) -> dict:
    """The reference's CPU path on the host cores, rank 0, N=1: the reference's
    FedAVGAlgorithm call sequence (oracle/ref_torch_cpu.py: process_worker_data per client with
    its torch CPU ops, then aggregate_worker_data) over ``n_clients`` pre-built messages of the
    headline workload (64 x ResNet-18 fp32, dataset-size weights). Timed in a fresh child process
    pinned to OMP_NUM_THREADS of the GPU's NUMA-local CPUs (the harness's per-GPU share) before
    torch starts its thread pool; the value is the best round, with min / median / max of the
    repeats and the host's load average beside it (the host is shared with other GPUs' jobs)."""
    import subprocess

    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    cpus, source = gpu_local_cpus(torch.cuda.current_device() if torch.cuda.is_available() else 0)
    pinned = cpus[:threads]
    spec = {"layout": next(k for k, f in LAYOUTS.items() if f().names == layout.names), "clients": n_clients,
            "dtype": str(dtype).split(".")[-1], "repeats": repeats, "budget_s": budget_s, "threads": threads,
            "cpus": pinned}
    load_parent = os.getloadavg()
    r = subprocess.run([sys.executable, str(REPO / "bench.py"), "--cpu-baseline-child", json.dumps(spec)],
                       capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        raise RuntimeError(f"cpu baseline child failed ({r.returncode}): {r.stderr[-2000:]}")
    res = json.loads(r.stdout.strip().splitlines()[-1])
    times = sorted(res["times_s"])
    best, med = times[0], times[len(times) // 2]
    nbytes = n_clients * layout.total_numel * dtype.itemsize + layout.total_numel * 4
    return {
        "value": round(nbytes / best / 1e9, 3),
        "unit": "GB/s",
        "cores": threads,
        "kind": "port",
        "host_cpu": host_cpu(),
        "seconds_per_round": round(best, 4),
        "repeats": {"n": len(times), "min_s": round(times[0], 4), "median_s": round(med, 4),
                    "max_s": round(times[-1], 4), "median_GBps": round(nbytes / med / 1e9, 3)},
        "pinning": {"cpus": pinned, "source": source, "threads_seen": res["threads_seen"]},
        "host_load": {"loadavg_1_5_15_before": [round(x, 2) for x in load_parent],
                      "loadavg_1_5_15_during": [round(x, 2) for x in res["loadavg_after"]],
                      "machine_cpus": os.cpu_count()},
        "sample": (
            f"the full round: {n_clients} pre-built ParameterMessages x {layout.num_segments}-tensor layout "
            f"({layout.total_numel:,} {str(dtype).split('.')[-1]} params), the reference's FedAVGAlgorithm call sequence "
            f"(process_worker_data x {n_clients}: isnan, to(f64)*w, +=; aggregate_worker_data: isnan, /W, isnan) "
            f"in torch CPU ops, best of {len(times)} in a child process pinned to {len(pinned)} CPUs ({source}), "
            f"{threads} threads ({res['wall_s']:.1f} s)"
        ),
    }


def cpu_baseline_personalized(layout: ModelLayout, budget_s: float = 12.0, workers: int = 5) -> dict:
    """The reference's PersonalizedFedAVG CPU op sequence on a bounded sample (rank 0, N=1)."""
    sys.path.insert(0, str(REPO))
    from oracle.ref_torch_cpu import RefOpsPersonalized

    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    torch.set_num_threads(threads)
    g = torch.Generator().manual_seed(1234)
    clients = [
        {n: torch.randn(s, generator=g, dtype=torch.float32) for n, s in zip(layout.names, layout.shapes)}
        for _ in range(workers)
    ]
    rng = np.random.default_rng(99)
    ww = {j: {i: float(rng.uniform(0.01, 3.0)) for i in range(workers) if i != j} for j in range(workers)}
    nbytes = workers * layout.total_numel * 4 + (workers + 1) * layout.total_numel * 8
    times = []
    t_start = time.perf_counter()
    while time.perf_counter() - t_start < budget_s and len(times) < 100:
        algo = RefOpsPersonalized(ww)
        t0 = time.perf_counter()
        for i, c in enumerate(clients):
            algo.add(i, c)
        algo.finish()
        times.append(time.perf_counter() - t0)
    best = min(times)
    return {
        "value": round(nbytes / best / 1e9, 3),
        "unit": "GB/s",
        "folds_per_s": round(workers * (workers - 1) * layout.total_numel / best, 1),
        "cores": threads,
        "kind": "port",
        "host_cpu": host_cpu(),
        "sample": (
            f"{workers} workers x {workers} receivers x ResNet-18 layout fp32, reference op sequence "
            "(deepcopy per receiver, isnan, to(f64)*w, +=, /W, isnan; centralized weighted_avg) in torch CPU, "
            f"best of {len(times)} runs over {time.perf_counter() - t_start:.1f} s"
        ),
    }


FP64_VALU_PEAK_TFLOPS = 78.6  # MI355X spec, vector fp64 (an FMA counts 2 flops)


def main_personalized(args: argparse.Namespace) -> int:
    """--workload personalized: one round of PersonalizedFedAVG (personalized_aggregation_algorithm.py),
    every worker a receiver (M = N = --clients-per-gpu), device-resident clients, one GPU."""
    from distributed_learning_simulation_lib_amd.personalized import PersonalizedContext, fp64_probe

    device = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
    torch.cuda.set_device(device)
    layout = LAYOUTS[args.layout]()
    P, N = layout.total_numel, args.clients_per_gpu
    M = N
    in_dtype = getattr(torch, args.in_dtype)
    out_dtype = torch.float64  # the reference's per-receiver models are float64
    _, views = make_clients(layout, 0, N, device, in_dtype)
    rng = np.random.default_rng(99)
    if args.pers_weights == "int":
        w = rng.integers(100, 5001, size=(M, N)).astype(np.float64)
    else:
        w = rng.uniform(0.01, 3.0, size=(M, N))
    ooffs, opad = layout.padded_offsets(8)
    out_bufs = [torch.empty(opad, dtype=out_dtype, device=device) for _ in range(M)]
    outs = [[b[o : o + n] for o, n in zip(ooffs, layout.numels)] for b in out_bufs]
    cbuf = torch.empty(opad, dtype=torch.float64, device=device)
    central = [cbuf[o : o + n] for o, n in zip(ooffs, layout.numels)]
    ctx = PersonalizedContext(layout, device)
    tables = ctx.tables(views, in_dtype, outs, out_dtype, central, torch.float64)
    ids = list(range(N))

    def step() -> None:
        ctx.aggregate(tables, in_dtype, ids, w, ids)
        if ctx.check():  # the reference's assertions: the round ends on the host
            raise AssertionError("NaN in a personalized aggregate")

    for _ in range(args.warmup):
        step()
    ctx.prof_enable(True)
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(device)
    elapsed = time.perf_counter() - t0
    kernel_ms, launches = ctx.prof_collect()
    step_s = elapsed / args.steps
    kstep_s = kernel_ms * 1e-3 / args.steps
    in_bytes = torch.empty((), dtype=in_dtype).element_size()
    job_bytes = N * P * in_bytes + M * P * 8 + P * 8
    folds = M * (N - 1) * P
    fused = args.pers_weights == "int"  # integer weights: every product exact -> one v_fma_f64 per fold
    lane_ops = folds * (1 if fused else 2) + 2 * M * P
    probe = None if args.no_probe else {"fp64_fma_TFLOPs": round(fp64_probe(device), 2), **hbm_probes(device)}
    cpu = None
    if not args.no_cpu_baseline:
        del views, tables
        torch.cuda.empty_cache()
        cpu = cpu_baseline_personalized(layout)
    short = {"float32": "fp32", "float16": "fp16", "bfloat16": "bf16", "float64": "fp64"}[args.in_dtype]
    line = {
        "metric": "PersonalizedFedAVG round, aggregated GB/s (device-resident)",
        "value": round(job_bytes / step_s / 1e9, 2),
        "unit": "GB/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(step_s * 1e3, 4),
        "higher_is_better": True,
        "scaling": "replicas only",
        "vs_baseline": None,
        "folds_per_s": round(folds / step_s, 1),  # (receiver, client, element) folds: the unit of work
        "dtype": "f64",
        "data": f"synthetic: client params ~ N(0,1), {args.pers_weights} weights (M x N)",
        "config": {"workload": f"personalized_fedavg_{args.layout}_{short}_{N}x{M}", "workers": N, "receivers": M,
                   "params_per_client": P, "tensors_per_client": layout.num_segments, "in_dtype": args.in_dtype,
                   "out_dtype": "float64", "fold": "fma (exact products)" if fused else "mul + add (rounded separately)"},
        "roofline": {
            "bound": "valu_fp64",
            "achieved": round(lane_ops / kstep_s / 1e12, 2),
            "peak": FP64_VALU_PEAK_TFLOPS / 2,
            "unit": "T fp64 VALU lane-ops/s",
            "frac": round(lane_ops / kstep_s / 1e12 / (FP64_VALU_PEAK_TFLOPS / 2), 4),
            "traffic": None,
            "kernel": "personalized_kernel<float, " + ("PF_FMA" if fused else "PF_MULADD") + ">",
            "kernel_ms_per_step": round(kstep_s * 1e3, 4),
            "launches": launches,
            "hbm_GBps": round(job_bytes / kstep_s / 1e9, 1),
        },
        "probe": probe,
        "cpu_baseline": cpu,
    }
    print(json.dumps(line), flush=True)
    return 0


def make_qsgd_clients(layout: ModelLayout, n: int, device: torch.device, level: int = 255, scheme: str = "qsgd"):
    """n synthetic quantised clients (fp32 codec), records resident in HBM: each client's
    x ~ N(0,1) (seeded per client) quantised with the client-side quantiser — QSGD
    (quantized.quantize_tensor, level 255: what a StochasticQuantClientEndpoint worker sends,
    quantized_endpoint.py:96-99) or NNADQ (quantized.nnadq_quantize_tensor, weight 0.01: an
    NNADQClientEndpoint worker, :114-124)."""
    from distributed_learning_simulation_lib_amd.quantized import (
        NNADQ_F32,
        nnadq_quantize_tensor,
        quantize_tensor,
        record_bytes,
    )

    sizes = [NNADQ_F32.record_bytes(m) if scheme == "nnadq" else record_bytes(m) for m in layout.numels]
    offs = np.cumsum([0] + sizes[:-1]).tolist()
    total = sum(sizes)
    buckets = torch.zeros((n, total), dtype=torch.uint8, device=device)
    g = torch.Generator(device=device)
    for i in range(n):
        g.manual_seed(1234 + i)
        for o, m, sz in zip(offs, layout.numels, sizes):
            x = torch.randn(m, generator=g, device=device)
            q = nnadq_quantize_tensor(x, NNADQ_WEIGHT) if scheme == "nnadq" else quantize_tensor(x, level, generator=g)
            buckets[i, o : o + sz] = q.record
    views = [[buckets[i, o : o + sz] for o, sz in zip(offs, sizes)] for i in range(n)]
    return buckets, views, total


NNADQ_WEIGHT = 0.01


def cpu_baseline_qsgd(layout: ModelLayout, budget_s: float = 12.0, sample_clients: int = 4) -> dict:
    """The reference's server path for quantised updates on the host: QuantServerEndpoint.get
    dequantises every tensor (x = norm * sign * slot / level in torch CPU ops,
    quantized_endpoint.py:69-77), then FedAVGAlgorithm's op sequence (oracle/ref_torch_cpu.py)."""
    sys.path.insert(0, str(REPO))
    from oracle.ref_torch_cpu import RefOpsFedAvg

    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    torch.set_num_threads(threads)
    weights = dataset_size_weights(sample_clients)
    g = torch.Generator().manual_seed(1234)
    clients = []
    for _ in range(sample_clients):
        c = {}
        for name, shape in zip(layout.names, layout.shapes):
            m = int(np.prod(shape))
            c[name] = (torch.rand((), generator=g).item() + 0.1,
                       torch.randint(0, 256, (m,), generator=g, dtype=torch.uint8),
                       torch.randint(0, 256, ((m + 7) // 8,), generator=g, dtype=torch.uint8), shape)
        clients.append(c)
    shifts = torch.arange(7, -1, -1, dtype=torch.uint8)
    rec_bytes = sum(m + (m + 7) // 8 for m in layout.numels)
    nbytes = sample_clients * rec_bytes + layout.total_numel * 4
    times = []
    t_start = time.perf_counter()
    while time.perf_counter() - t_start < budget_s and len(times) < 1000:
        algo = RefOpsFedAvg()
        t0 = time.perf_counter()
        for c, w in zip(clients, weights):
            dense = {}
            for name, (norm, slots, packed, shape) in c.items():
                sign = ((packed.unsqueeze(1) >> shifts) & 1).reshape(-1)[: slots.numel()].to(torch.float32) * 2 - 1
                dense[name] = ((torch.tensor(norm, dtype=torch.float32) * sign) * slots.to(torch.float32) / 255).view(shape)
            algo.add(dense, w)
        out = {k: v.to(torch.float32) for k, v in algo.finish().items()}
        times.append(time.perf_counter() - t0)
    best = min(times)
    return {
        "value": round(nbytes / best / 1e9, 3),
        "unit": "GB/s",
        "cores": threads,
        "kind": "port",
        "host_cpu": host_cpu(),
        "sample": (
            f"{sample_clients} QSGD-quantised clients x ResNet-18 layout (fp32 codec, level 255): host "
            f"dequantisation (unpack signs, norm * sign * slot / level) + the reference FedAvg op sequence "
            f"in torch CPU, best of {len(times)} runs over {time.perf_counter() - t_start:.1f} s"
        ),
    }


def cpu_baseline_nnadq(layout: ModelLayout, budget_s: float = 12.0, sample_clients: int = 4) -> dict:
    """The reference's server path for NNADQ updates on the host: QuantServerEndpoint.get
    dequantises every tensor (x = code * step + lo in torch CPU ops, quantized_endpoint.py:69-77,
    127-136), then FedAVGAlgorithm's op sequence (oracle/ref_torch_cpu.py)."""
    sys.path.insert(0, str(REPO))
    from oracle.ref_torch_cpu import RefOpsFedAvg

    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    torch.set_num_threads(threads)
    weights = dataset_size_weights(sample_clients)
    g = torch.Generator().manual_seed(1234)
    clients = []
    for _ in range(sample_clients):
        c = {}
        for name, shape in zip(layout.names, layout.shapes):
            m = int(np.prod(shape))
            c[name] = (torch.rand((), generator=g).item() - 0.5, torch.rand((), generator=g).item() * 1e-2,
                       torch.randint(0, 201, (m,), generator=g, dtype=torch.uint8), shape)
        clients.append(c)
    nbytes = sample_clients * sum(32 + m for m in layout.numels) + layout.total_numel * 4
    times = []
    t_start = time.perf_counter()
    while time.perf_counter() - t_start < budget_s and len(times) < 1000:
        algo = RefOpsFedAvg()
        t0 = time.perf_counter()
        for c, w in zip(clients, weights):
            dense = {name: (codes.to(torch.float32) * step + lo).view(shape)
                     for name, (lo, step, codes, shape) in c.items()}
            algo.add(dense, w)
        out = {k: v.to(torch.float32) for k, v in algo.finish().items()}
        times.append(time.perf_counter() - t0)
    best = min(times)
    return {
        "value": round(nbytes / best / 1e9, 3),
        "unit": "GB/s",
        "cores": threads,
        "kind": "port",
        "host_cpu": host_cpu(),
        "sample": (
            f"{sample_clients} NNADQ-quantised clients x ResNet-18 layout (fp32 codec): host dequantisation "
            f"(code * step + lo) + the reference FedAvg op sequence in torch CPU, best of {len(times)} runs "
            f"over {time.perf_counter() - t_start:.1f} s"
        ),
    }


def main_qsgd(args: argparse.Namespace) -> int:
    """--workload qsgd: one FedAvg round over QSGD-quantised client updates (the server behind
    StochasticQuantServerEndpoint, quantized_endpoint.py:102-111) with the dequantisation fused
    into the fold; records resident in HBM, one GPU."""
    from distributed_learning_simulation_lib_amd.quantized import NNADQ_F32, QSGD_F32

    nnadq = args.workload == "nnadq"
    fmt = NNADQ_F32 if nnadq else QSGD_F32
    device = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
    torch.cuda.set_device(device)
    layout = LAYOUTS[args.layout]()
    P, T, N = layout.total_numel, layout.num_segments, args.clients_per_gpu
    out_dtype = getattr(torch, args.out_dtype)
    buckets, views, client_bytes = make_qsgd_clients(layout, N, device, scheme="nnadq" if nnadq else "qsgd")
    weights = dataset_size_weights(N)
    table = ClientTable(T)
    for row, w in zip(views, weights):
        table.add_client(row, [w] * T)
    ctx = FedAvgContext(layout, device)
    offs, padded = layout.padded_offsets(torch.empty((), dtype=out_dtype).element_size())
    out_flat = torch.empty(padded, dtype=out_dtype, device=device)
    outs = OutputTable([out_flat[o : o + m] for o, m in zip(offs, layout.numels)], layout, device, out_dtype)
    plan = ctx.plan(table, fmt, outs, out_dtype)

    def step() -> None:
        plan.run()
        ctx.raise_on_nan()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(device)
    ctx.prof_collect()
    ctx.prof_enable(True)
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(device)
    elapsed = time.perf_counter() - t0
    ctx.prof_enable(False)
    kernel_ms, launches = ctx.prof_collect()
    out_bytes = torch.empty((), dtype=out_dtype).element_size()
    job_bytes = N * client_bytes + P * out_bytes  # every record byte the fold must read + the result
    step_s = elapsed / args.steps
    per_launch_s = kernel_ms * 1e-3 / max(launches, 1)
    achieved = job_bytes / per_launch_s / 1e9
    probe = None if args.no_probe else hbm_probes(device)
    traffic, traffic_src = None, None
    # the newest PMC pass of this line's kernel (QSGD: round 4's XCD-contiguous placement)
    cands = sorted((REPO / "profiles").glob(f"r[0-9][0-9]_traffic_{'nnadq' if nnadq else 'qsgd'}.json"))
    tfile = cands[-1] if cands else REPO / "profiles" / "missing.json"
    if tfile.exists() and N == 64 and args.layout == "resnet18" and out_dtype == torch.float32:
        traffic = float(json.loads(tfile.read_text())["hbm_traffic_bytes_per_step"])
        traffic_src = f"profiles/{tfile.name}"
    cpu = None
    if not args.no_cpu_baseline:
        del buckets, views, table, plan
        torch.cuda.empty_cache()
        cpu = cpu_baseline_nnadq(layout) if nnadq else cpu_baseline_qsgd(layout)
    line = {
        "metric": ("aggregated GB/s (device-resident), N-client weighted FedAvg reduce over "
                   f"{'NNADQ' if nnadq else 'QSGD'}-quantised updates"),
        "value": round(job_bytes / step_s / 1e9, 2),
        "unit": "GB/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(step_s * 1e3, 4),
        "higher_is_better": True,
        "scaling": "replicas only",
        "vs_baseline": None,
        "client_elements_per_s": round(N * P / step_s, 1),
        "dtype": "f64",
        "data": ("synthetic: x ~ N(0,1) per client, " + (
            f"NNADQ-quantised on the GPU (deterministic, weight {NNADQ_WEIGHT})" if nnadq else
            "QSGD-quantised on the GPU (inf-norm, level 255, stochastic rounding)") + "; dataset-size weights"),
        "config": {"workload": f"fedavg_{'nnadq' if nnadq else 'qsgd255'}_{args.layout}_{N}_clients", "clients": N,
                   "params_per_client": P, "tensors_per_client": T, "record_bytes_per_client": client_bytes,
                   "codec": "nnadq_f32" if nnadq else "qsgd_f32 (level 255)",
                   "accumulate_dtype": "float64", "out_dtype": args.out_dtype},
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 4),
            "traffic": traffic,
            "traffic_source": traffic_src,
            "kernel": (f"{'nnadq' if nnadq else 'qsgd'}_tile_kernel<OUT_{'F32' if out_dtype == torch.float32 else 'F64'}, "
                       f"float{', fma' if nnadq else ''}, true>"),
            "bytes_per_launch": job_bytes,
            "mean_launch_ms": round(per_launch_s * 1e3, 4),
            "launches": launches,
        },
        "hbm_probe": probe,
        "cpu_baseline": cpu,
    }
    if not nnadq:
        # the |product| tables qsgd_table_kernel builds per launch (K clients x 256 fp64 per segment,
        # launches split at FEDAVG_QSGD_TABLE_CAP, 64 MiB by default): written once and read by the
        # fold, so ~2x these bytes of traffic ride on top of bytes_per_launch
        cap = int(os.environ.get("FEDAVG_QSGD_TABLE_CAP", 64 << 20))
        per_seg = N * 256 * 8
        line["roofline"]["qsgd_table_bytes"] = min(T, max(1, cap // per_seg)) * per_seg
    print(json.dumps(line), flush=True)
    return 0


def main_plugin(args: argparse.Namespace) -> int:
    """--workload plugin: the drop-in path the reference's server drives
    (aggregation_server.py:111-145): FedAVGAlgorithm.process_worker_data x N + aggregate_worker_data
    + clear_worker_data per round on one long-lived algorithm object, N device-resident updates of
    named tensors (--clients-per-gpu, ResNet-18 by default), the reference's fp64 result left on the
    device. Each round's messages are built inside its step, as the server receives them (the
    payload tensors stay resident; ~0.4 us per message, reported within host_us_per_update)."""
    from distributed_learning_simulation_lib_amd import FedAVGAlgorithm, ParameterMessage

    device = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
    torch.cuda.set_device(device)
    layout = LAYOUTS[args.layout]()
    P, T, N = layout.total_numel, layout.num_segments, args.clients_per_gpu
    in_dtype = getattr(torch, args.in_dtype)
    out_dtype = getattr(torch, args.out_dtype)
    buckets, views = make_clients(layout, 0, N, device, in_dtype)
    params = [{n: v.view(s) for n, s, v in zip(layout.names, layout.shapes, row)} for row in views]
    weights = dataset_size_weights(N)
    algo = FedAVGAlgorithm(device=device, wave_size=args.wave if args.wave > 0 else None, result_dtype=out_dtype,
                           wave_min=args.wave_min if args.wave_min >= 0 else None)
    wave = min(algo.wave_size, N)  # the plugin's own default unless --wave is given

    # --workload gradient: GradientWorker._process_gradient's message every step (gradient_worker.py:
    # 83-93): the native-dtype gradient dict, in_round=True, the dataset size as weight
    in_round = args.workload == "gradient"

    def messages():
        # one message at a time, as the server receives them (each is handed over on arrival)
        return (ParameterMessage(parameter=dict(p), aggregation_weight=w, in_round=in_round)
                for p, w in zip(params, weights))

    host_s = [0.0]
    # --arrival bursts:K:GAP_MS — the reference server's cadence (server.py:133-146): it polls every
    # worker, hands what arrived to the algorithm back to back, then sleeps; here K bursts of N/K
    # updates with GAP_MS of host time between them. The latency its loop sees is the last
    # arrival -> the result (aggregate_worker_data returning on the host).
    bursts, gap_s = 1, 0.0
    if args.arrival != "all":
        kind, k_s, g_s = args.arrival.split(":")
        assert kind == "bursts", args.arrival
        bursts, gap_s = int(k_s), float(g_s) / 1e3
        assert 1 <= bursts <= N and N % bursts == 0, "bursts must divide the clients"
    per_burst = N // bursts
    tail_s = [0.0]

    def step() -> None:
        h0 = time.perf_counter()
        for wid, m in enumerate(messages()):
            if wid and wid % per_burst == 0 and gap_s:
                time.sleep(gap_s)
            algo.process_worker_data(wid, m)
        t_last = time.perf_counter()
        host_s[0] += t_last - h0
        res = algo.aggregate_worker_data()  # ends on the host: the NaN flags are read (:93, :97)
        tail_s[0] += time.perf_counter() - t_last
        algo.clear_worker_data()
        assert len(res.parameter) == T and res.in_round == in_round

    for _ in range(args.warmup):
        step()
    ctx = algo._context()
    ctx.prof_collect()
    ctx.prof_enable(not args.no_kernel_events)
    host_s[0] = 0.0
    tail_s[0] = 0.0
    dyn0 = dict(algo.dyn_stats)
    ctx.dyn_prof_collect()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(device)
    elapsed = time.perf_counter() - t0
    ctx.prof_enable(False)
    kernel_ms, launches = ctx.prof_collect()
    dyn_ms, dyn_waves = ctx.dyn_prof_collect()
    dyn = {k: round((algo.dyn_stats[k] - dyn0[k]) / args.steps, 2) for k in dyn0}
    host_timed, tail_timed = host_s[0], tail_s[0]
    if dyn_waves and not args.no_kernel_events:
        # after the timed region: the same rounds again, each wave's tiles recording when they
        # finished (fedavg_dyn_timing, GPU clock): the fold after the last rows reached the tiles
        # (result stores included) and after the close, medians over the rounds
        dyn_t: dict[str, list[float]] = {"rows_to_end_us": [], "close_to_end_us": []}
        ctx.prof_enable(True)
        for _ in range(min(args.steps, 10)):
            step()
            tm = algo._context().dyn_timing()
            for key in dyn_t:
                if tm[key] >= 0:
                    dyn_t[key].append(tm[key])
        ctx.prof_enable(False)
        ctx.prof_collect()
        ctx.dyn_prof_collect()
        host_s[0], tail_s[0] = host_timed, tail_timed  # the timed rounds' host times only
        for key, vals in dyn_t.items():
            dyn[key.replace("_us", "_ms_median")] = round(float(np.median(vals)) / 1e3, 4) if vals else None
    in_b, out_b = in_dtype.itemsize, out_dtype.itemsize
    job_bytes = N * P * in_b + P * out_b
    n_waves = -(-N // wave)
    if algo.wave_min and launches and not args.no_kernel_events:
        n_waves = max(1, round(launches / args.steps))  # early waves: the launches that ran
    launch_bytes = job_bytes + (n_waves - 1) * P * 16  # + the fp64 accumulator round trips between waves
    step_s = elapsed / args.steps
    kstep_s = kernel_ms * 1e-3 / args.steps
    achieved = launch_bytes / kstep_s / 1e9 if kstep_s > 0 else 0.0
    dyn_rows_all = dyn_waves and dyn["rows"] == N and dyn["finalized"] == 1
    if dyn_rows_all:
        # every row folded by the round's dynamic wave: its body launch (enqueue at the first
        # arrival to its end, arrival phase included) carries the round's bytes
        kstep_s = dyn_ms * 1e-3 / args.steps
        launch_bytes = job_bytes
        achieved = launch_bytes / kstep_s / 1e9 if kstep_s > 0 else 0.0
    # the HBM probes (read / copy ceilings; their known byte counts calibrate a PMC pass's
    # FETCH_SIZE / WRITE_SIZE in the same process, scripts/dyn_traffic.sh)
    probe = None if args.no_probe else hbm_probes(device)
    burst = None
    if bursts > 1:
        # one burst's clients folded by the one-launch kernel (HIP events): the fold time the
        # burst's latency is judged against (last arrival -> result <= 1.2x of it)
        bctx = FedAvgContext(layout, device)
        btab = ClientTable(T)
        for row, w in zip(views[-per_burst:], weights[-per_burst:]):
            btab.add_client(row, [w] * T)
        offs_b, pad_b = layout.padded_offsets(out_b)
        bflat = torch.empty(pad_b, dtype=out_dtype, device=device)
        bouts = OutputTable([bflat[o : o + n] for o, n in zip(offs_b, layout.numels)], layout, device, out_dtype)
        bplan = bctx.plan(btab, in_dtype, bouts, out_dtype)
        for _ in range(3):
            bplan.run()
        bctx.raise_on_nan()
        bctx.prof_collect()
        bctx.prof_enable(True)
        for _ in range(10):
            bplan.run()
        bctx.raise_on_nan()
        bctx.prof_enable(False)
        b_ms, b_n = bctx.prof_collect()
        del bplan
        bctx.close()
        burst_ms = b_ms / max(b_n, 1)
        lat_ms = tail_s[0] / args.steps * 1e3
        burst = {"bursts": bursts, "updates_per_burst": per_burst, "gap_ms": gap_s * 1e3,
                 "last_arrival_to_result_ms": round(lat_ms, 4),
                 "one_burst_fold_ms": round(burst_ms, 4),
                 "ratio": round(lat_ms / burst_ms, 3) if burst_ms else None,
                 "what": "last process_worker_data returned -> aggregate_worker_data returned (result on the "
                         "device, NaN flags read), against one burst's clients folded and divided by the "
                         "one-launch kernel (fedavg_tile_kernel, HIP events)"}
    cpu = None
    if not args.no_cpu_baseline:
        del params, views, buckets
        algo.exit()
        torch.cuda.empty_cache()
        cpu = cpu_baseline(layout, n_clients=N, dtype=in_dtype)
        if in_round:  # the same round, as a latency
            cpu = dict(cpu, value=round(cpu["seconds_per_round"] * 1e3, 3), unit="ms per round")
    short = {"float32": "fp32", "float16": "fp16", "bfloat16": "bf16", "float64": "fp64"}[args.in_dtype]
    gbps = round(job_bytes / step_s / 1e9, 2)
    workload = (f"{'gradient' if in_round else 'plugin'}_fedavg_{args.layout}_{short}_{N}_clients"
                + (f"_in_{bursts}_bursts_{gap_s * 1e3:g}ms_apart" if bursts > 1 else "")
                + (f"_waves_of_{wave}" if n_waves > 1 and not algo.wave_min else "")
                + (f"_early_waves_from_{algo.wave_min}" if algo.wave_min else ""))
    traffic, traffic_ratio, traffic_src = committed_dyn_traffic(workload) if dyn_rows_all else (None, None, None)
    line = {
        "metric": ("burst-cadence FedAvg round through the plugin surface (the reference server's poll-then-sleep "
                   "loop): last arrival to result latency" if burst else
                   "in-round gradient FedAvg round latency (GradientWorker cadence) through the plugin surface: "
                   "FedAVGAlgorithm.process_worker_data x N + aggregate_worker_data" if in_round else
                   "aggregated GB/s (device-resident) through the plugin surface: FedAVGAlgorithm."
                   "process_worker_data x N + aggregate_worker_data"),
        **({"burst_arrivals": burst} if burst else {}),
        "value": (burst["last_arrival_to_result_ms"] if burst else round(step_s * 1e3, 4) if in_round else gbps),
        "unit": "ms last arrival to result" if burst else "ms per round" if in_round else "GB/s",
        "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(step_s * 1e3, 4), "higher_is_better": not (in_round or burst),
        "scaling": "replicas only", "vs_baseline": None, "dtype": "f64", "GBps": gbps,
        "data": "synthetic: client params ~ N(0,1) seeded per client, weights = dataset sizes in [100, 5000]",
        "config": {"workload": workload,
                   "clients": N, "params_per_client": P, "tensors_per_client": T, "in_dtype": args.in_dtype,
                   "out_dtype": args.out_dtype, "clients_per_launch": wave, "wave_min": algo.wave_min,
                   "waves_per_round": round(launches / args.steps, 2) if launches else None, "in_round": in_round,
                   # the round's first wave folded during the arrivals (fedavg_dyn_*):
                   # rows it folded and rounds it divided itself, per round; its kernel spans the
                   # arrival phase, so the event timing and roofline below cover the ordinary waves only
                   "dynamic_wave": dict(dyn, enabled=algo.dynamic_wave),
                   "host_us_per_update": round(host_s[0] / (args.steps * N) * 1e6, 2),
                   "process_worker_data_ms_per_round": round(host_s[0] / args.steps * 1e3, 4),
                   # what a round costs beyond its kernels: staging, launch, NaN readback, result dict
                   "fixed_ms_per_round": round((step_s - kstep_s) * 1e3, 4),
                   "baseline_config": ("GradientWorker in-round rounds (gradient_worker.py:83-93), see DESIGN.md §4"
                                       if in_round else
                                       "BASELINE.json configs[1] through the reference's plugin call sequence")},
        "roofline": {
            "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic, "traffic_over_algorithmic": traffic_ratio,
            "traffic_source": traffic_src,
            "kernel": ("dyn_wave_kernel (body launch, enqueued at the first arrival; arrivals included)"
                       if dyn_rows_all else f"fedavg_tile_kernel x {n_waves} launch(es) per round"),
            "bytes_per_step": launch_bytes,
            "kernel_ms_per_step": round(kstep_s * 1e3, 4), "launches": launches + dyn_waves},
        "hbm_probe": probe,
        "cpu_baseline": cpu,
    }
    print(json.dumps(line), flush=True)
    return 0


SPEEDUP_TARGET = {4: 3.5}  # BASELINE.json north_star: >= 3.5x at 4 GPUs (strong scaling, config 3)


def one_gpu_anchor(layout: ModelLayout, n_total: int, weights: list, in_dtype: torch.dtype, out_dtype: torch.dtype,
                   device: torch.device, steps: int, warmup: int, resident: list | None = None) -> dict:
    """The same n_total-client job on ``device`` alone with the N = 1 fused kernel, timed like the
    one-GPU line (one plan launch + the NaN readback per round, bench.py --gpus 1 --total-clients
    n_total): the anchor of an N > 1 line's measured speed-up, taken in the same run. ``resident``:
    (first client, row views) already on ``device`` (the shard of entry 0, or every shard of an
    aliased rehearsal); the other clients are generated there from their seeds."""
    T = layout.num_segments
    have = {first + i: row for first, views in (resident or []) for i, row in enumerate(views)}
    made, rows, c = [], [], 0
    while c < n_total:
        if c in have:
            rows.append(have[c])
            c += 1
            continue
        stop = c
        while stop < n_total and stop not in have:
            stop += 1
        buckets, views = make_clients(layout, c, stop - c, device, in_dtype)
        made.append(buckets)
        rows.extend(views)
        c = stop
    table = ClientTable(T)
    for row, w in zip(rows, weights):
        table.add_client(row, [w] * T)
    ctx = FedAvgContext(layout, device)
    offs, padded = layout.padded_offsets(out_dtype.itemsize)
    flat = torch.empty(padded, dtype=out_dtype, device=device)
    outs = OutputTable([flat[o : o + n] for o, n in zip(offs, layout.numels)], layout, device, out_dtype)
    reducer = HipLocalReducer(ctx, table, in_dtype, outs, out_dtype)

    def step() -> None:
        reducer.fused()
        reducer.raise_on_nan()

    for _ in range(warmup):
        step()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize(device)
    ms = (time.perf_counter() - t0) / steps * 1e3
    generated = sum(b.numel() * b.element_size() for b in made)
    del reducer, table, made, rows
    ctx.close()
    torch.cuda.empty_cache()
    return {"anchor_ms_per_step": round(ms, 4), "anchor_device": str(device), "anchor_clients": n_total,
            "anchor_clients_generated_bytes": generated}


def speedup_block(G: int, ms_per_step: float | None, anchor: dict | None, aliased: bool,
                  tail: tuple[float, float, int] | None = None, predicted: dict | None = None) -> dict:
    """The N > 1 line's own verdict on the north-star speed-up: the same-N one-GPU anchor timed in
    this run, measured_speedup = anchor / ms_per_step, the target for this G, and the exposed
    exchange tail measured with events beside the cost model's. An aliased rehearsal (every entry
    on one GPU) reports its ratio as ``aliased_ratio`` only: it is not a scaling figure."""
    a = None if anchor is None else anchor["anchor_ms_per_step"]
    ratio = None if a is None or not ms_per_step else round(a / ms_per_step, 3)
    target = SPEEDUP_TARGET.get(G)
    out = {"anchor": anchor, "measured_speedup": None if aliased else ratio,
           "aliased_ratio": ratio if aliased else None, "target_speedup": target,
           "meets_target": None if aliased or ratio is None or target is None else bool(ratio >= target),
           "basis": ("aliased rehearsal: every entry on one GPU, not a scaling figure" if aliased else
                     "measured: the same clients on device 0 alone vs this line's step, one run")}
    if tail is not None:
        fold, tl, n = tail
        out["events"] = {"rounds": n, "entry0_fold_ms": None if not n else round(fold / n, 4),
                         "exposed_exchange_and_finalize_ms": None if not n else round(tl / n, 4),
                         "predicted_exposed_exchange_and_finalize_ms":
                             None if predicted is None else predicted.get("exposed_exchange_and_finalize_ms"),
                         "what": "entry 0's stream: round start -> its last chunk fold -> the round's end behind "
                                 "every exchange (fedavg_multi_prof_*), over rounds after the timed ones"}
    return out


def main_multi(args: argparse.Namespace) -> int:
    """--procs 1 --gpus N: ONE process drives N GPUs through the single-process multi-device mode
    (include/fedavg_hip.h fedavg_multi_*) — the structure of the reference's single
    server process (simulation_lib/server/server.py:122-152). BASELINE config 3 (256 clients,
    contiguous shards), the peer-window exchange (or --multi-exchange reduce: in-process RCCL); the
    (exchange, chunks, shape) candidate is timed on the node before the warmup (--tune-budget),
    or taken from the cost model with --no-tune. --alias: every entry on cuda:0 (a one-GPU code-path
    rehearsal, not an N-GPU measurement)."""
    from distributed_learning_simulation_lib_amd.multi_device import MultiDeviceContext

    G = args.gpus
    _STAGES.start(0, args.stage_timeout, "peer" if args.multi_exchange == "peer" else "native")
    _STAGES.enter("create")
    _inject_failure("one_process")
    devices = [0] * G if args.alias else list(range(G))
    if not args.alias and torch.cuda.device_count() < G:
        print(f"bench.py --procs 1 --gpus {G}: only {torch.cuda.device_count()} GPU(s) visible "
              "(--alias rehearses)", file=sys.stderr)
        return 3
    in_dtype, out_dtype = getattr(torch, args.in_dtype), getattr(torch, args.out_dtype)
    layout = LAYOUTS[args.layout]()
    P, T = layout.total_numel, layout.num_segments
    n_total = job_clients(args, G)
    weights_all = dataset_size_weights(n_total)
    m = MultiDeviceContext(layout, devices)
    if args.multi_exchange == "peer" and not m.peer_access:
        print(f"bench.py --procs 1: no peer access between the devices {devices}; the peer exchange "
              "cannot run", file=sys.stderr)
        m.close()
        return 3
    _STAGES.enter("make_clients")
    keep, tables, rows_of = [], [], []
    for g, d in enumerate(devices):
        lo, hi = shard_bounds(n_total, G, g)
        dev = torch.device("cuda", d)
        buckets, views = make_clients(layout, lo, hi - lo, dev, in_dtype)
        keep.append(buckets)
        rows_of.append((lo, views))
        t = ClientTable(T)
        for row, w in zip(views, weights_all[lo:hi]):
            t.add_client(row, [w] * T)
        tables.append(t if hi > lo else None)
    _STAGES.enter("plan")
    partials = m.plan_partials(tables, in_dtype)
    root_dev = torch.device("cuda", devices[0])
    offs, padded = layout.padded_offsets(out_dtype.itemsize)
    out_flat = torch.empty(padded, dtype=out_dtype, device=root_dev)
    outs = OutputTable([out_flat[o : o + n] for o, n in zip(offs, layout.numels)], layout, root_dev, out_dtype)
    W = -0.0
    for w in weights_all:
        W += w
    totals = [W] * T
    nt = m.num_tiles
    model = ExchangeModel()
    in_b, out_b = in_dtype.itemsize, out_dtype.itemsize
    exchanges = (args.multi_exchange,)
    cands = exchange_candidates(args.chunks or None, exchanges=exchanges)
    pending = [[(t, in_dtype)] if t is not None else [] for t in tables]

    def sync_all() -> None:
        for d in sorted(set(devices)):
            torch.cuda.synchronize(d)

    def one_round(ex: str, edges: list[int]) -> None:
        # a round ends as the server's does, on the host: the NaN flags of every entry are read
        # once the round's end event completed (one wait, like the one-GPU line's stream sync)
        m.round(partials, totals, outs, out_dtype, root=0, edges=edges, exchange=ex)
        m.raise_on_nan(pending, round_only=True)

    tuned, selection = None, "cost model"
    _STAGES.enter("tune", args.tune_budget + args.stage_timeout)
    if args.no_tune:
        (ex, ch, sh), _ = model.best(G, P, n_total, in_b, out_b, nt, cands, balance_root=False)
    else:
        times, t_start = {}, time.perf_counter()
        for cand in cands:
            e = chunk_edges(nt, cand[1], cand[2])
            one_round(cand[0], e)
            sync_all()
            t0 = time.perf_counter()
            for _ in range(3):
                one_round(cand[0], e)
            sync_all()
            times[cand] = (time.perf_counter() - t0) / 3 * 1e3
            if time.perf_counter() - t_start > args.tune_budget:
                break
        ex, ch, sh = min(times, key=lambda c: (times[c], cands.index(c)))
        tuned = {f"{a}/{b}/{c}": round(v, 4) for (a, b, c), v in times.items()}
        selection = "tuned"
    edges = chunk_edges(nt, ch, sh)
    _STAGES.enter("warmup")
    for _ in range(args.warmup):
        one_round(ex, edges)
    sync_all()
    _STAGES.enter("timed")
    t0 = time.perf_counter()
    for _ in range(args.steps):
        one_round(ex, edges)
    sync_all()
    elapsed = time.perf_counter() - t0
    step_s = elapsed / args.steps
    job_bytes = n_total * P * in_b + P * out_b
    value = job_bytes / step_s / 1e9

    # the result of the last timed round, sampled, against host fp64 compositions of the same
    # clients (and every client row against its regeneration from its seed)
    _STAGES.enter("result_check")
    picks = sample_elements(layout)
    got = out_flat[flat_index(layout, picks, out_b, root_dev)].to(torch.float64).cpu().numpy()
    shards, shard_w, changed = [], [], 0
    for g, d in enumerate(devices):
        lo, hi = shard_bounds(n_total, G, g)
        s, c = gather_client_samples(keep[g], flat_index(layout, picks, in_b, torch.device("cuda", d)), lo)
        shards.append(s)
        shard_w.append(weights_all[lo:hi])
        changed += c
    check = result_check(got, shards, shard_w, args.out_dtype, "composition" if ex == "peer" else None)
    check["client_rows_changed"] = changed
    check["ok"] = check["ok"] and changed == 0

    # the dominant kernel, after the timed region: entry 0's windowed partial launches (one per
    # chunk) timed with HIP events on its stream over the same number of rounds
    _STAGES.enter("kernel_events")
    ctx0 = m.contexts[0]
    ctx0.prof_collect()
    ctx0.prof_enable(not args.no_kernel_events)
    for _ in range(args.steps):
        one_round(ex, edges)
    sync_all()
    ctx0.prof_enable(False)
    kernel_ms, launches = ctx0.prof_collect()
    lo0, hi0 = shard_bounds(n_total, G, 0)
    rank_bytes = P * (hi0 - lo0) * in_b + P * 8  # its clients' reads + its fp64 partial stores (local or peer)
    kernel_step_ms = kernel_ms / args.steps
    achieved = rank_bytes / (kernel_step_ms * 1e-3) / 1e9 if kernel_ms > 0 else 0.0
    predicted = model.round_ms(G, P, n_total, in_b, out_b, edges, ex) if G > 1 else None
    one_gpu = model.one_gpu_ms(P, n_total, in_b, out_b)
    # the exposed exchange + division tail, event-timed on entry 0 over the same number of rounds
    _STAGES.enter("exchange_tail")
    m.prof_collect()
    m.prof_enable(True)
    for _ in range(args.steps):
        one_round(ex, edges)
    sync_all()
    m.prof_enable(False)
    tail = m.prof_collect()
    _STAGES.enter("teardown")
    m.close()
    del partials
    # the same N-client job on device 0 alone, N = 1 kernel, same steps and warmup
    _STAGES.enter("anchor", args.stage_timeout + 120)
    anchor = None if args.no_anchor else one_gpu_anchor(
        layout, n_total, weights_all, in_dtype, out_dtype, root_dev, args.steps, args.warmup,
        resident=[r for g, r in enumerate(rows_of) if devices[g] == devices[0]])
    speed = speedup_block(G, step_s * 1e3, anchor, args.alias, tail, predicted)
    _STAGES.enter("done", 0)
    line = {
        "metric": METRIC, "value": round(value, 2), "unit": "GB/s", "n_gpus": len(set(devices)), "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(step_s * 1e3, 4), "higher_is_better": True,
        "scaling": "weak" if args.weak else "strong", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic: client params ~ N(0,1) seeded per client, weights = dataset sizes in [100, 5000]",
        "config": {
            "workload": workload_name(args, G, n_total, 1, n_total // G) + "_one_process",
            "total_clients": n_total, "device_entries": devices, "params_per_client": P, "tensors_per_client": T,
            "in_dtype": args.in_dtype, "accumulate_dtype": "float64", "out_dtype": args.out_dtype,
            "parallelism": f"one process, {G} device entries: clients sharded, "
                           + ("peer-window exchange over xGMI (fedavg_multi_round)" if ex == "peer"
                              else "in-process RCCL reduce (fedavg_multi_round)"),
            "launch": {"mode": "one process driving every GPU (bench.py --procs 1)",
                       "launched_by": os.environ.get("BENCH_LAUNCHED_BY", "none"),
                       "round_check": "per round: one event wait behind every entry's exchange, then the NaN "
                                      "flags (fedavg_multi_round_check)"},
            "exchange": {"mode": ex, "chunks": ch, "chunk_shape": sh, "selection": selection,
                         "tuned_ms_per_round": tuned,
                         "predicted_speedup": None if predicted is None else predicted["speedup"],
                         "predicted": predicted, "one_gpu_model_ms": round(one_gpu, 4)},
            "baseline_config": "BASELINE.json configs[2] driven from one process" if n_total == 256 else "see DESIGN.md",
            **({"rehearsal": f"all {G} entries on cuda:0: a code-path check of the exchange, not an N-GPU measurement"}
               if args.alias else {}),
        },
        "roofline": {
            "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": None,
            "kernel": f"fedavg_tile_kernel<{args.in_dtype}, OUT_ACC, windowed> on entry 0 (its chunk launches)",
            "bytes_per_step_this_rank": rank_bytes, "kernel_ms_per_step": round(kernel_step_ms, 4),
            "launches": launches,
        },
        "speedup": speed,
        "result_check": check,
        "cpu_baseline": None,
    }
    if not check["ok"]:
        # not on stdout: a fallback run prints the job's one line
        print(f"bench.py --procs 1: the result check failed; the line was: {json.dumps(line)}", file=sys.stderr,
              flush=True)
        return 3
    print(json.dumps(line), flush=True)
    return 0


def main_elements(args: argparse.Namespace) -> int:
    """--shard elements: every rank folds its element range of ALL clients (range_sharded.py):
    bit-identical to one GPU at any N, the exchange is a gather of the fp32 result. The same
    256-client job as BASELINE config 3, decomposed by elements instead of by clients."""
    from distributed_learning_simulation_lib_amd.range_sharded import RangeShard, range_sharded_reduce

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    device = torch.device("cuda", 0 if args.rehearse else local_rank)
    torch.cuda.set_device(device)
    if world > 1:
        _rendezvous_env()
        if args.rehearse:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        else:
            dist.init_process_group("nccl", device_id=device, rank=rank, world_size=world)
    in_dtype, out_dtype = getattr(torch, args.in_dtype), getattr(torch, args.out_dtype)
    layout = LAYOUTS[args.layout]()
    P = layout.total_numel
    n_total = args.total_clients if args.total_clients > 0 else (256 if world > 1 else args.clients_per_gpu)
    weights = dataset_size_weights(n_total)
    shard = RangeShard(layout, world, rank, device)
    T = len(shard.pieces)
    table = None
    buckets = None
    if T:
        buckets, views = make_clients(shard.sub_layout, 0, n_total, device, in_dtype)
        table = ClientTable(T)
        for row, w in zip(views, weights):
            table.add_client(row, [w] * T)
    out = torch.empty(P, dtype=out_dtype, device=device) if rank == 0 else None

    def step() -> None:
        range_sharded_reduce(shard, table, in_dtype, out, out_dtype)

    def sync_all() -> None:
        torch.cuda.synchronize(device)
        if dist.is_initialized():
            dist.barrier()
        torch.cuda.synchronize(device)

    for _ in range(args.warmup):
        step()
    sync_all()
    if shard.ctx is not None:
        shard.ctx.prof_collect()
        shard.ctx.prof_enable(not args.no_kernel_events)
    sync_all()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    sync_all()
    elapsed = time.perf_counter() - t0
    kernel_ms, launches = (0.0, 0)
    if shard.ctx is not None:
        shard.ctx.prof_enable(False)
        kernel_ms, launches = shard.ctx.prof_collect()
    if dist.is_initialized():
        t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if args.rehearse else device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        dist.barrier()
        dist.destroy_process_group()
    if rank != 0:
        return 0
    in_b, out_b = torch.empty((), dtype=in_dtype).element_size(), torch.empty((), dtype=out_dtype).element_size()
    step_s = elapsed / args.steps
    job_bytes = n_total * P * in_b + P * out_b
    span = shard.hi - shard.lo
    launch_bytes = n_total * span * in_b + span * out_b
    per_launch = kernel_ms / max(launches, 1)
    achieved = launch_bytes / (per_launch * 1e-3) / 1e9 if launches else 0.0
    short = {"float32": "fp32", "float16": "fp16", "bfloat16": "bf16", "float64": "fp64"}[args.in_dtype]
    kname = {torch.float32: "float", torch.float16: "__half", torch.bfloat16: "bf16_t", torch.float64: "double"}[in_dtype]
    line = {
        "metric": METRIC, "value": round(job_bytes / step_s / 1e9, 2), "unit": "GB/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(step_s * 1e3, 4),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic: client params ~ N(0,1) seeded per client, weights = dataset sizes in [100, 5000]",
        "config": {
            "workload": f"fedavg_{args.layout}_{short}_{n_total}_clients_element_ranges_over_{world}_gpus",
            "total_clients": n_total, "params_per_client": P, "tensors_per_client": layout.num_segments,
            "in_dtype": args.in_dtype, "accumulate_dtype": "float64", "out_dtype": args.out_dtype,
            "parallelism": f"element ranges over {world} GPUs (every rank folds its range of all clients, "
                           "bit-identical to one GPU) + gather of the result to rank 0",
            "rank0_range": [shard.lo, shard.hi],
            "baseline_config": "BASELINE.json configs[2] job, decomposed by element range (see DESIGN.md §5d)",
            **({"rehearsal": "all ranks on cuda:0 over gloo: a code-path check, not an N-GPU measurement"}
               if args.rehearse else {}),
        },
        "roofline": {
            "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": None, "traffic_source": None,
            "kernel": f"fedavg_tile_kernel<{kname}, OUT_F32, 1, true, fma> (rank 0's range)",
            "bytes_per_timed_launch": launch_bytes, "kernel_ms_per_step": round(kernel_ms / args.steps, 4),
            "mean_launch_ms": round(per_launch, 4), "launches": launches,
        },
        "cpu_baseline": None,
    }
    print(json.dumps(line), flush=True)
    del buckets
    return 0


def committed_traffic(world: int, n_local: int, in_dtype: str, out_dtype: str) -> tuple[float | None, str | None]:
    """HBM bytes per launch of the same kernel and workload from the newest committed
    rocprofv3 PMC summary (scripts/profile.sh -> profiles/<tag>_traffic.json), or None."""
    if world != 1 or n_local != 64 or in_dtype != "float32" or out_dtype != "float32":
        return None, None
    files = sorted((REPO / "profiles").glob("r[0-9][0-9]_traffic.json"))  # not the per-config r*_traffic_cfg*
    if not files:
        return None, None
    d = json.loads(files[-1].read_text())
    return float(d["hbm_traffic_bytes_per_launch"]), f"profiles/{files[-1].name}"


def committed_dyn_traffic(workload: str) -> tuple[float | None, float | None, str | None]:
    """(HBM bytes per round, ratio to algorithmic, source) of the dynamic wave for this plugin /
    gradient workload from the newest committed PMC summary (scripts/dyn_traffic.sh ->
    profiles/<tag>_dyn_traffic_<name>.json), or Nones."""
    for f in sorted((REPO / "profiles").glob("r[0-9][0-9]_dyn_traffic_*.json"), reverse=True):
        d = json.loads(f.read_text())
        if d.get("workload") == workload and d.get("hbm_traffic_bytes_per_round"):
            return float(d["hbm_traffic_bytes_per_round"]), round(float(d["traffic_over_algorithmic"]), 4), \
                f"profiles/{f.name}"
    return None, None, None


def job_clients(args: argparse.Namespace, world: int) -> int:
    """Clients of the whole job: BASELINE.json configs[2] (256 over the GPUs) at N > 1, configs[1]
    (--clients-per-gpu = 64) on one GPU; --weak keeps --clients-per-gpu on every rank."""
    if args.weak:
        return args.clients_per_gpu * world
    if args.total_clients > 0:
        return args.total_clients
    return 256 if world > 1 else args.clients_per_gpu


def shard_bounds(n_total: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous client shards: rank r folds clients [lo, hi) (N/G each; the dispatcher's split)."""
    return rank * n_total // world, (rank + 1) * n_total // world


def workload_name(args: argparse.Namespace, world: int, n_total: int, n_waves: int, wave: int) -> str:
    short = {"float32": "fp32", "float16": "fp16", "bfloat16": "bf16", "float64": "fp64"}[args.in_dtype]
    name = f"fedavg_{args.layout}_{short}_{n_total}_clients"
    if world > 1:
        name += f"_sharded_over_{world}_gpus" + ("_weak" if args.weak else "")
    if n_waves > 1:
        name += f"_waves_of_{wave}"
    return name


def _rendezvous_env() -> None:
    """MASTER_ADDR / MASTER_PORT for a process group: the launcher's (or torchrun's) when set,
    else 127.0.0.1 and a free port (a one-rank --force-collective run)."""
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if "MASTER_PORT" not in os.environ:
        os.environ["MASTER_PORT"] = str(_free_port())


def _inject_failure(where: str) -> None:
    """Test hook: BENCH_INJECT_FAIL=<where> makes that path exit with status 3 (the launcher's
    fallback tests)."""
    if os.environ.get("BENCH_INJECT_FAIL") == where:
        print(f"bench.py: injected failure in the {where} run", file=sys.stderr, flush=True)
        raise SystemExit(3)


def main_dry_one_process(args: argparse.Namespace) -> int:
    """--dry-run --procs 1 --gpus N: the single-process skeleton of main_multi on the CPU — stage
    watchdog, client shards of the N device entries, the peer schedule of the cost model."""
    G = args.gpus
    _STAGES.start(0, args.stage_timeout, "peer")
    _STAGES.enter("create")
    _inject_failure("one_process")
    layout = LAYOUTS[args.layout]()
    n_total = job_clients(args, G)
    shards = [list(shard_bounds(n_total, G, g)) for g in range(G)]
    _STAGES.enter("timed")
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pass
    _ = time.perf_counter() - t0
    model = ExchangeModel()
    nt = -(-layout.total_numel // 4096)  # a 4096-element tile count of the order of the library's
    (ex, ch, sh), pred = model.best(G, layout.total_numel, n_total, 4, 4, nt,
                                    exchange_candidates(exchanges=("peer",)), balance_root=False)
    _STAGES.enter("done", 0)
    line = {
        "metric": METRIC, "value": None, "unit": "GB/s", "n_gpus": G, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": None, "higher_is_better": True,
        "scaling": "weak" if args.weak else "strong", "vs_baseline": None, "dtype": "f64",
        "data": "dry run: no client data, no GPU work",
        "config": {"workload": workload_name(args, G, n_total, 1, n_total // G) + "_one_process",
                   "total_clients": n_total, "params_per_client": layout.total_numel,
                   "tensors_per_client": layout.num_segments, "client_shards": shards,
                   "launch": {"mode": "one process", "devices": G},
                   "exchange": {"mode": ex, "chunks": ch, "chunk_shape": sh, "selection": "cost model",
                                "predicted_speedup": pred["speedup"]},
                   "launched_by": os.environ.get("BENCH_LAUNCHED_BY", "none")},
        "speedup": speedup_block(G, None, None, args.alias, (0.0, 0.0, 0), pred),
        "dry_run": "launcher check on the CPU: the single-process run's skeleton; not a measurement",
    }
    print(json.dumps(line), flush=True)
    return 0


def main_dry(args: argparse.Namespace) -> int:
    """--dry-run: the multi-rank skeleton of main() on the CPU — gloo group, client shards, a
    barrier-bracketed timed region of empty steps, max over ranks, one JSON line from rank 0."""
    if args.procs == 1 and args.gpus > 1:
        return main_dry_one_process(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        _STAGES.start(rank, args.stage_timeout, args.comm)
        _STAGES.enter("init_process_group")
        _rendezvous_env()
        dist.init_process_group("gloo", rank=rank, world_size=world, timeout=timedelta(seconds=PG_TIMEOUT_S))
        _STAGES.enter("shards")
    layout = LAYOUTS[args.layout]()
    n_total = job_clients(args, world)
    lo, hi = shard_bounds(n_total, world, rank)
    if hi - lo < 1:
        raise SystemExit(f"{n_total} clients cannot be sharded over {world} ranks")
    wave = args.wave if 0 < args.wave < hi - lo else hi - lo
    n_waves = -(-(hi - lo) // wave)
    shards = torch.tensor([lo, hi], dtype=torch.int64)
    if world > 1:
        gathered = [torch.empty(2, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(gathered, shards)
        dist.barrier()
    else:
        gathered = [shards]
    if world > 1:
        _STAGES.enter("timed")
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pass
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.barrier()
        dist.destroy_process_group()
    if rank != 0:
        return 0
    line = {
        "metric": METRIC, "value": None, "unit": "GB/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": None, "higher_is_better": True,
        "scaling": "weak" if args.weak else "strong", "vs_baseline": None, "dtype": "f64",
        "data": "dry run: no client data, no GPU work",
        "config": {"workload": workload_name(args, world, n_total, n_waves, wave), "total_clients": n_total,
                   "params_per_client": layout.total_numel, "tensors_per_client": layout.num_segments,
                   "client_shards": [[int(a), int(b)] for a, b in (g.tolist() for g in gathered)],
                   "launched_by": os.environ.get("BENCH_LAUNCHED_BY", "external launcher" if world > 1 else "none")},
        "dry_run": "launcher check on the CPU: rank processes, gloo group, shards, max-over-ranks timing; "
                   "not a measurement",
    }
    if world > 1:
        line["speedup"] = speedup_block(world, None, None, args.rehearse)
    if os.environ.get("BENCH_LAUNCH_FALLBACK"):
        line["config"]["launch_fallback"] = os.environ["BENCH_LAUNCH_FALLBACK"]
    print(json.dumps(line), flush=True)
    return 0


def _one_process_under_launcher(args: argparse.Namespace) -> bool:
    """The default (``--procs 0``) under an external launcher (torch.distributed.run: WORLD_SIZE set,
    every rank of one node): rank 0 drives every GPU in one process, as the self-launcher's child."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    return (args.procs == 0 and world > 1 and world == args.gpus and args.workload == "fedavg"
            and args.shard == "clients" and not args.rehearse
            and int(os.environ.get("LOCAL_WORLD_SIZE", str(world))) == world
            # the ranks meet on torch.distributed.run's own store (no process group is created here,
            # so the per-process fallback can still create its own)
            and os.environ.get("TORCHELASTIC_USE_AGENT_STORE") == "True")


def main_one_process_under_launcher(args: argparse.Namespace) -> int | None:
    """torch.distributed.run form of the default launch: rank 0 runs the single-process multi-device
    round (main_multi: every GPU of the node, peer exchange) while the other ranks wait on
    torch.distributed.run's own store for its exit status (no process group: the fallback below
    creates the job's one). 0: rank 0 printed the job's line and every rank exits
    0. Otherwise (no peer access, a failed result check, an error) every rank returns None and the
    same processes run the per-process path (fresh process group; rank 0 closed its multi-device
    object; no process is re-executed), the line saying so in config.launch_fallback."""
    world = int(os.environ["WORLD_SIZE"])
    rank = int(os.environ.get("RANK", "0"))
    budget = args.one_process_timeout + 60.0
    store = dist.PrefixStore("bench_one_process", dist.TCPStore(
        os.environ["MASTER_ADDR"], int(os.environ["MASTER_PORT"]), world, is_master=False,
        timeout=timedelta(seconds=budget)))
    status = torch.tensor([1], dtype=torch.int64)
    if rank == 0:
        os.environ.setdefault("BENCH_LAUNCHED_BY", "torch.distributed.run (rank 0 drives every GPU)")
        one = argparse.Namespace(**vars(args))
        one.procs = 1
        try:
            rc = main_dry_one_process(one) if args.dry_run else main_multi(one)
        except SystemExit as e:
            rc = e.code if isinstance(e.code, int) else 1
        except Exception as e:  # noqa: BLE001 - any failure of the one-process run falls back
            import traceback

            traceback.print_exc()
            print(f"bench.py rank 0: the one-process run raised {type(e).__name__}: {e}", file=sys.stderr)
            rc = 1
        status[0] = int(rc or 0)
        store.set("status", str(int(status.item())))
    else:
        store.wait(["status"])
        status[0] = int(store.get("status").decode())
    if int(status.item()) == 0:
        return 0
    note = (f"the single-process peer run on rank 0 failed (status {int(status.item())}); this line is the "
            "per-process run of the same torch.distributed.run ranks")
    os.environ["BENCH_LAUNCH_FALLBACK"] = note
    os.environ.pop("BENCH_LAUNCHED_BY", None)
    if rank == 0:
        print(f"bench.py: {note}", file=sys.stderr, flush=True)
        if not args.dry_run:
            import gc

            gc.collect()  # the one-process run's client buffers and receive slots, on every device
            for d in range(torch.cuda.device_count()):
                with torch.cuda.device(d):
                    torch.cuda.empty_cache()
    return None


def main() -> int:
    if len(sys.argv) == 3 and sys.argv[1] == "--cpu-baseline-child":
        print(json.dumps(_cpu_baseline_child(json.loads(sys.argv[2]))), flush=True)
        return 0
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--layout", default="resnet18", choices=sorted(LAYOUTS))
    ap.add_argument("--clients-per-gpu", type=int, default=None,
                    help="weak scaling (--weak) and the personalized / qsgd workloads: clients per GPU")
    ap.add_argument("--total-clients", type=int, default=0,
                    help="clients of the whole job, sharded over the ranks (0 = auto: --clients-per-gpu "
                         "(64) on one GPU = BASELINE config 2; 256 on N > 1 GPUs = BASELINE config 3, "
                         "strong scaling)")
    ap.add_argument("--weak", action="store_true",
                    help="weak scaling instead: --clients-per-gpu clients on every rank")
    ap.add_argument("--wave", type=int, default=0, help="clients per launch (streaming waves); 0 = all")
    ap.add_argument("--wave-min", type=int, default=-1,
                    help="plugin early waves: fold >= this many staged clients whenever the GPU is idle "
                         "(0 = full waves only; -1 = the plugin's default)")
    ap.add_argument("--chunks", type=int, default=0,
                    help="tile chunks of the sharded reduce (0 = auto: 4 when world > 1 — "
                         "the RCCL reduce of chunk c overlaps the partial of chunk c+1, DESIGN.md §5)")
    ap.add_argument("--comm", default="native", choices=["native", "torch"],
                    help="sharded path: the library's own RCCL communicator, whole round in one native "
                         "call (native) or the chunks' reduces through torch.distributed (torch)")
    ap.add_argument("--exchange", default="auto", choices=["auto", "reduce", "scatter"],
                    help="multi-GPU exchange of the fp64 partials: reduce to rank 0, or reduce-scatter + "
                         "per-rank finalize + gather (auto: the fastest (exchange, chunks) pair timed on the "
                         "node before the warmup; with --no-tune scatter at 2 ranks, reduce above; DESIGN.md §5)")
    ap.add_argument("--shard", default="clients", choices=["clients", "elements"],
                    help="N > 1: shard whole clients over the ranks (BASELINE config 3, default) or "
                         "element ranges of every client (range_sharded.py: bit-identical to one GPU)")
    ap.add_argument("--rehearse", action="store_true",
                    help="N > 1 on a one-GPU box: all ranks on cuda:0 over gloo (host-staged exchange); "
                         "exercises the multi-rank code path, not a measurement")
    ap.add_argument("--no-tune", action="store_true",
                    help="N > 1 with --exchange auto: take the cost model's exchange instead of timing "
                         "every (exchange, chunks) candidate before the warmup")
    ap.add_argument("--in-dtype", default="float32", choices=["float32", "float16", "bfloat16", "float64"])
    ap.add_argument("--out-dtype", default=None, choices=["float32", "float64"],
                    help="result dtype (default float32; float64 — the reference's — for --workload plugin)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-probe", action="store_true")
    ap.add_argument("--no-kernel-events", action="store_true",
                    help="diagnostic: time the steps without per-launch HIP events (no roofline)")
    ap.add_argument("--no-plan", action="store_true", help="re-stage the client table every round")
    ap.add_argument("--force-collective", action="store_true",
                    help="one GPU: run the sharded path (partial + RCCL reduce + finalize) anyway")
    ap.add_argument("--workload", default="fedavg", choices=["fedavg", "personalized", "qsgd", "nnadq", "plugin", "gradient"],
                    help="fedavg: the headline reduce; personalized: PersonalizedFedAVG (one GPU); "
                         "qsgd / nnadq: FedAvg over QSGD- / NNADQ-quantised updates, dequantisation fused (one GPU); "
                         "plugin: the headline round through FedAVGAlgorithm's plugin calls (one GPU); "
                         "gradient: GradientWorker's in-round rounds through the plugin, as a latency "
                         "(--clients-per-gpu default 8)")
    ap.add_argument("--pers-weights", default="float", choices=["float", "int"])
    ap.add_argument("--arrival", default="all",
                    help="--workload plugin / gradient: 'all' (updates back to back) or bursts:K:GAP_MS — K "
                         "bursts with GAP_MS of host time between them (the reference server's poll-then-sleep "
                         "cadence); the line then reports last_arrival_to_result_ms")
    ap.add_argument("--launch-timeout", type=float, default=480.0,
                    help="--gpus N > 1 without an external launcher: seconds before the spawned ranks are "
                         "stopped and the run fails (one --comm torch rerun within the same budget)")
    ap.add_argument("--no-fallback", action="store_true",
                    help="self-launched N > 1: no --comm torch rerun after a failed native-communicator run")
    ap.add_argument("--stage-timeout", type=float, default=150.0,
                    help="N > 1: a rank whose current stage (init, comm, tune, warmup, timed, ...) runs longer "
                         "ends with status 124, naming the stage (0 = no watchdog)")
    ap.add_argument("--tune-budget", type=float, default=60.0,
                    help="N > 1 with --exchange auto: seconds of exchange tuning before the best candidate "
                         "timed so far is taken")
    ap.add_argument("--procs", type=int, default=0,
                    help="--gpus N > 1: 1 = one process drives the N GPUs (fedavg_multi_*, the single-process "
                         "multi-device mode, peer-window exchange); N = one rank process per GPU (RCCL); "
                         "0 (default) = the one-process run, and fresh per-process ranks if it fails")
    ap.add_argument("--one-process-timeout", type=float, default=200.0,
                    help="--gpus N > 1 (default launch): seconds the one-process run may take before the "
                         "launcher stops it and starts the per-process ranks (capped at half --launch-timeout)")
    ap.add_argument("--no-anchor", action="store_true",
                    help="N > 1: skip timing the same-N job on GPU 0 alone after the timed region (the "
                         "line's measured_speedup is then null)")
    ap.add_argument("--alias", action="store_true",
                    help="--procs 1: every device entry on cuda:0 (a one-GPU rehearsal of the multi-device round)")
    ap.add_argument("--multi-exchange", default="peer", choices=["peer", "reduce"],
                    help="--procs 1: the peer-window exchange (no collective library) or the in-process RCCL reduce")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher check without a GPU: every rank joins a gloo group, takes its client "
                         "shard and the max-over-ranks timing of an empty step; prints the JSON line "
                         "with value null (no measurement)")
    args = ap.parse_args()
    if args.out_dtype is None:
        args.out_dtype = "float64" if args.workload in ("plugin", "gradient") else "float32"
    if args.clients_per_gpu is None:
        args.clients_per_gpu = 8 if args.workload == "gradient" else 64
    if _one_process_under_launcher(args):
        rc = main_one_process_under_launcher(args)
        if rc is not None:
            return rc
        args.procs = args.gpus  # the one-process run failed: this rank continues per process
    if args.dry_run:
        return main_dry(args)
    if args.workload == "personalized":
        return main_personalized(args)
    if args.workload in ("qsgd", "nnadq"):
        return main_qsgd(args)
    if args.workload in ("plugin", "gradient"):
        return main_plugin(args)
    if args.shard == "elements":
        return main_elements(args)
    if args.procs == 1 and args.gpus > 1:
        return main_multi(args)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    # --rehearse: every rank on cuda:0 over a gloo group (the exchange staged through host memory,
    # RCCL refuses two ranks on one GPU) — runs this N > 1 code path on a one-GPU box; its times
    # are not the N-GPU numbers
    if world > 1:
        _STAGES.start(rank, args.stage_timeout, args.comm)
        _STAGES.enter("init_process_group")
    device = torch.device("cuda", 0 if args.rehearse else local_rank)
    torch.cuda.set_device(device)
    pg_timeout = timedelta(seconds=PG_TIMEOUT_S)
    if args.rehearse and (world > 1 or args.force_collective):
        _rendezvous_env()
        dist.init_process_group("gloo", rank=rank, world_size=world, timeout=pg_timeout)
        args.comm = "torch"
    elif world > 1 or args.force_collective:
        _rendezvous_env()
        # RCCL on a high-priority stream: its workgroups take free CU slots ahead of the next
        # chunk's partial-kernel workgroups, so the reduce of chunk c starts under chunk c+1
        opts = dist.ProcessGroupNCCL.Options()
        opts.is_high_priority_stream = True
        dist.init_process_group("nccl", device_id=device, rank=rank, world_size=world, pg_options=opts,
                                timeout=pg_timeout)
    if world > 1:
        _STAGES.enter("make_clients")
    sharded = world > 1 or args.force_collective
    chunks_auto = args.chunks <= 0
    if chunks_auto:
        args.chunks = 4 if world > 1 else 2

    in_dtype = getattr(torch, args.in_dtype)
    out_dtype = getattr(torch, args.out_dtype)
    layout = LAYOUTS[args.layout]()
    P = layout.total_numel
    T = layout.num_segments
    n_total = job_clients(args, world)
    lo, hi = shard_bounds(n_total, world, rank)
    n_local = hi - lo
    if n_local < 1:
        raise SystemExit(f"{n_total} clients cannot be sharded over {world} ranks")
    wave = args.wave if 0 < args.wave < n_local else n_local
    weights_all = dataset_size_weights(n_total)
    my_weights = weights_all[lo:hi]

    buckets, views = make_clients(layout, lo, n_local, device, in_dtype)
    tables = []
    for w0 in range(0, n_local, wave):
        t = ClientTable(T)
        for row, w in zip(views[w0 : w0 + wave], my_weights[w0 : w0 + wave]):
            t.add_client(row, [w] * T)
        tables.append(t)
    ctx = FedAvgContext(layout, device)
    outs = None
    if rank == 0:
        offs, padded = layout.padded_offsets(torch.empty((), dtype=out_dtype).element_size())
        out_flat = torch.empty(padded, dtype=out_dtype, device=device)
        outs = OutputTable([out_flat[o : o + m] for o, m in zip(offs, layout.numels)], layout, device, out_dtype)
    reducer = HipLocalReducer(ctx, tables[-1], in_dtype, outs, out_dtype, prior_waves=tables[:-1],
                              use_plan=not args.no_plan)
    local_totals = [float(sum(my_weights))] * T
    global_totals = [float(sum(weights_all))] * T

    host_enqueue = [0.0]  # host time to enqueue one round (diagnostic: is the step host-bound?)

    comm = None
    if world > 1:
        _STAGES.enter("comm_create")
    if sharded and args.comm == "native":
        try:
            comm = RcclComm(device)
        except Exception as e:  # e.g. no RCCL symbols: the same schedule through torch.distributed
            print(f"warning: native RCCL communicator unavailable ({e}); using --comm torch", file=sys.stderr)
            args.comm = "torch"

    exchange = resolve_exchange(args.exchange, world)
    selection = "fixed" if args.exchange != "auto" else "cost model"
    tuned = None
    chunk_shape = "even"
    model = ExchangeModel()
    in_b, out_b = in_dtype.itemsize, out_dtype.itemsize
    if sharded and world > 1 and args.exchange == "auto" and args.no_tune:
        # DESIGN.md §5 cost model: the (exchange, chunks, shape) with the smallest predicted step
        (exchange, ch, chunk_shape), _ = model.best(
            world, P, n_total, in_b, out_b, ctx.num_tiles, exchange_candidates(None if chunks_auto else args.chunks),
            balance_root=False)
        args.chunks = ch
    if sharded and args.exchange == "auto" and not args.no_tune:
        # time every (exchange, chunks) candidate on this node before the warmup (untimed; the
        # max over ranks decides, so every rank picks the same): the link rate the DESIGN.md §5
        # cost model assumes is not measurable on one GPU
        if world > 1:
            _STAGES.enter("tune", args.tune_budget + args.stage_timeout)
        (exchange, args.chunks, chunk_shape), times = tune_exchange(
            reducer, local_totals, exchange_candidates(None if chunks_auto else args.chunks), rounds=3,
            global_total_weights=global_totals, comm=comm, force_collective=args.force_collective,
            budget_s=args.tune_budget)
        tuned = {f"{e}/{c}/{sh}": round(ms, 4) for (e, c, sh), ms in times.items()}
        selection = "tuned"

    def step() -> None:
        h0 = time.perf_counter()
        # rank 0 ends the round on the host: sharded_reduce reads the NaN flags there (the
        # reference's assertions, fed_avg_algorithm.py:35,93,97)
        sharded_reduce(reducer, local_totals, chunks=args.chunks, global_total_weights=global_totals,
                       force_collective=args.force_collective, comm=comm, exchange=exchange, check_nan=False,
                       shape=chunk_shape)
        host_enqueue[0] += time.perf_counter() - h0
        if rank == 0:
            reducer.raise_on_nan()

    if world > 1:
        _STAGES.enter("warmup")
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(device)
    if dist.is_initialized():
        dist.barrier()
    if world > 1:
        _STAGES.enter("timed")
    ctx.prof_collect()  # drop warmup events
    host_enqueue[0] = 0.0
    ctx.prof_enable(not args.no_kernel_events)
    torch.cuda.synchronize(device)
    if dist.is_initialized():
        dist.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(device)
    if dist.is_initialized():
        dist.barrier()
    torch.cuda.synchronize(device)
    elapsed = time.perf_counter() - t0
    ctx.prof_enable(False)
    kernel_ms, launches = ctx.prof_collect()
    if dist.is_initialized():
        t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if args.rehearse else device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    in_bytes = torch.empty((), dtype=in_dtype).element_size()
    out_bytes = torch.empty((), dtype=out_dtype).element_size()
    # the result of the last timed round, sampled (every tensor's ends + 4096 random elements),
    # against host fp64 compositions of the same clients; every client row is also compared with
    # its regeneration from its seed. Rank 0 checks; the other ranks send their shards' samples.
    if world > 1:
        _STAGES.enter("result_check")
    picks = sample_elements(layout)
    s_local, changed = gather_client_samples(buckets, flat_index(layout, picks, in_bytes, device), lo)
    bounds = [shard_bounds(n_total, world, r) for r in range(world)]
    if dist.is_initialized():
        xdev = torch.device("cpu") if args.rehearse else device
        n_max = max(b - a for a, b in bounds)
        mine = torch.zeros((n_max, len(picks)), dtype=torch.float64, device=xdev)
        mine[:n_local] = torch.from_numpy(s_local).to(xdev)
        every = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(every, mine)
        ch = torch.tensor([changed], dtype=torch.int64, device=xdev)
        dist.all_reduce(ch)
        changed = int(ch.item())
        shard_samples = [every[r][: b - a].cpu().numpy() for r, (a, b) in enumerate(bounds)]
    else:
        shard_samples = [s_local]
    check = None
    if rank == 0:
        got = out_flat[flat_index(layout, picks, out_bytes, device)].to(torch.float64).cpu().numpy()
        check = result_check(got, shard_samples, [weights_all[a:b] for a, b in bounds], args.out_dtype,
                             "single" if world == 1 else None)
        check["client_rows_changed"] = changed
        check["ok"] = check["ok"] and changed == 0

    job_bytes = n_total * P * in_bytes + P * out_bytes
    step_s = elapsed / args.steps
    value_gbps = job_bytes / step_s / 1e9

    n_local_max = max(((r + 1) * n_total // world) - (r * n_total // world) for r in range(world))
    # dominant kernel family, per step on this rank: the client reads + the result write
    # (fused single launch) or + the fp64 partial/accumulator traffic (waves, shards)
    n_waves = len(tables)
    rank_bytes = n_local * P * in_bytes
    if not sharded:
        rank_bytes += P * out_bytes + (n_waves - 1) * P * 16  # fp64 accumulator round trips between waves
    else:
        rank_bytes += (n_waves - 1) * P * 16 + P * 8 + (P * (8 + out_bytes) if rank == 0 else 0)
    kernel_step_s = kernel_ms * 1e-3 / args.steps
    achieved = rank_bytes / kernel_step_s / 1e9 if kernel_step_s > 0 else 0.0
    per_launch_ms = kernel_ms / max(launches, 1)
    kname = {torch.float32: "float", torch.float16: "__half", torch.bfloat16: "bf16_t", torch.float64: "double"}[in_dtype]
    kernel_desc = None
    if comm is not None and n_waves == 1:
        # native round: one timed launch per round, the first chunk's partial kernel (events
        # around every chunk would put markers into the pipeline they measure)
        a, b = ctx.tile_range(0, chunk_edges(ctx.num_tiles, args.chunks, chunk_shape)[1])
        rank_bytes = (b - a) * (n_local * in_bytes + 8)
        achieved = rank_bytes / (per_launch_ms * 1e-3) / 1e9 if launches else 0.0
        kernel_desc = f"fedavg_tile_kernel<{kname}, OUT_ACC, 1, true, fma> (partial, first of {args.chunks} chunks)"

    # Diagnostic for the sharded round (untimed, after the timed region): the same number of
    # partial-only rounds (the chunk kernels without the exchange), so the line shows how much
    # of the step is the exposed reduce tail + the root's finalize.
    partial_only_ms = None
    pplan = getattr(reducer, "_partial_plan", None) if sharded else None
    if world > 1:
        _STAGES.enter("partial_only")
    if pplan is not None:
        torch.cuda.synchronize(device)
        if dist.is_initialized():
            dist.barrier()
        torch.cuda.synchronize(device)
        p0 = time.perf_counter()
        for _ in range(args.steps):
            pplan.run()
        torch.cuda.synchronize(device)
        p_el = time.perf_counter() - p0
        if dist.is_initialized():
            pt = torch.tensor([p_el], dtype=torch.float64, device="cpu" if args.rehearse else device)
            dist.all_reduce(pt, op=dist.ReduceOp.MAX)
            p_el = float(pt.item())
        partial_only_ms = p_el / args.steps * 1e3

    # N > 1: the same N-client job on rank 0's GPU alone (N = 1 kernel, same steps and warmup),
    # timed in this run while the other ranks wait, so the line carries its own measured speed-up
    anchor = None
    if world > 1 and not args.no_anchor:
        _STAGES.enter("anchor", args.stage_timeout + 120)
        torch.cuda.synchronize(device)
        if rank == 0:
            anchor = one_gpu_anchor(layout, n_total, weights_all, in_dtype, out_dtype, device, args.steps,
                                    args.warmup, resident=[(lo, views)])
        if dist.is_initialized():
            dist.barrier()

    traffic, traffic_src = (None, None)
    if not sharded and n_waves == 1 and args.layout == "resnet18":
        traffic, traffic_src = committed_traffic(world, n_local, args.in_dtype, args.out_dtype)
    probe = None
    cpu = None
    if rank == 0 and not args.no_probe:
        probe = hbm_probes(device)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        del buckets, views, tables, reducer
        torch.cuda.empty_cache()
        cpu = cpu_baseline(layout)

    if world > 1:
        _STAGES.enter("teardown")
    if comm is not None:
        torch.cuda.synchronize(device)
        comm.close()
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()
    if world > 1:
        _STAGES.enter("done", 0)
    if rank != 0:
        return 0
    workload = workload_name(args, world, n_total, n_waves, wave)
    predicted = None if world < 2 else model.round_ms(
        world, P, n_total, in_b, out_b, chunk_edges(ctx.num_tiles, args.chunks, chunk_shape), exchange)
    # the single-process peer exchange (--procs 1) at its best schedule, for comparison
    peer_cand, peer_pred = (None, None) if world < 2 else model.best(
        world, P, n_total, in_b, out_b, ctx.num_tiles, candidates=exchange_candidates(exchanges=("peer",)))
    if args.layout == "resnet18" and not args.weak and n_total == 64 and world == 1:
        baseline_config = "BASELINE.json configs[1]"
    elif args.layout == "resnet18" and not args.weak and n_total == 256:
        baseline_config = ("BASELINE.json configs[2] (256 clients sharded over the GPUs, strong scaling)" if world > 1
                           else "BASELINE.json configs[2] on one GPU (the same-N anchor of the 2/4/8-GPU lines)")
    elif args.layout == "resnet18" and args.weak:
        baseline_config = f"BASELINE.json configs[2] weak-scaled ({n_local} clients per GPU)"
    else:
        baseline_config = "see DESIGN.md"
    line = {
        "metric": METRIC,
        "value": round(value_gbps, 2),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(step_s * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak" if args.weak else "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic: client params ~ N(0,1) seeded per client, weights = dataset sizes in [100, 5000]",
        "config": {
            "workload": workload,
            "clients_per_gpu": n_local_max,
            "total_clients": n_total,
            "clients_per_launch": wave,
            "client_table": "re-staged every round" if args.no_plan else "prepared once (persistent client slots)",
            "params_per_client": P,
            "tensors_per_client": T,
            "in_dtype": args.in_dtype,
            "accumulate_dtype": "float64",
            "out_dtype": args.out_dtype,
            "parallelism": "single GPU" if world == 1 else (
                f"clients sharded over {world} GPUs + chunked RCCL "
                + ("reduce to rank 0" if exchange == "reduce" else "reduce-scatter, per-rank finalize, gather to rank 0")),
            "exchange": None if not sharded else {
                "mode": exchange, "chunks": args.chunks, "chunk_shape": chunk_shape, "comm": args.comm,
                "selection": selection,
                "tuned_ms_per_round": tuned,
                "partial_only_ms_per_step": None if partial_only_ms is None else round(partial_only_ms, 4),
                "exposed_exchange_and_finalize_ms": (None if partial_only_ms is None
                                                     else round(step_s * 1e3 - partial_only_ms, 4)),
                # DESIGN.md §5 cost model for this schedule (measured one-GPU rates, quoted xGMI
                # rate x assumed RCCL efficiency): its fold / exposed terms beside the measured ones
                "predicted_speedup": None if predicted is None else predicted["speedup"],
                "predicted": predicted,
                "peer_mode_predicted_speedup": None if peer_pred is None else peer_pred["speedup"],
                "peer_mode_predicted": None if peer_pred is None else dict(peer_pred, schedule=list(peer_cand)),
            },
            "baseline_config": baseline_config,
            **({"rehearsal": "all ranks on cuda:0 over gloo: a code-path check, not an N-GPU measurement"}
               if args.rehearse else {}),
            **({"launch_fallback": os.environ["BENCH_LAUNCH_FALLBACK"]} if os.environ.get("BENCH_LAUNCH_FALLBACK")
               else {}),
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 4),
            "traffic": traffic,
            "traffic_source": traffic_src,
            "kernel": kernel_desc or (f"fedavg_tile_kernel<{kname}, OUT_F32, 1, true, fma>" if not sharded and n_waves == 1
                       else f"fedavg_tile_kernel<{kname}, ...> x {n_waves} waves" + (" + RCCL reduce + finalize" if sharded else "")),
            "bytes_per_timed_launch" if kernel_desc else "bytes_per_step_this_rank": rank_bytes,
            "kernel_ms_per_step": round(kernel_ms / args.steps, 4),
            "mean_launch_ms": round(per_launch_ms, 4),
            "launches": launches,
        },
        # the input-only form N·P·s_in / t beside the algorithmic-bytes value
        "input_only_GBps": round(n_total * P * in_bytes / step_s / 1e9, 2),
        **({"speedup": speedup_block(world, step_s * 1e3, anchor, args.rehearse, None, predicted)}
           if world > 1 else {}),
        "host_enqueue_ms_per_step": round(host_enqueue[0] * 1e3 / args.steps, 4),
        "hbm_probe": probe,
        "result_check": check,
        "cpu_baseline": cpu,
    }
    if world > 1:
        line["config"]["launch"] = {"mode": f"one process per GPU ({world} ranks, torch.distributed)",
                                    "launched_by": os.environ.get("BENCH_LAUNCHED_BY", "external launcher")}
    print(json.dumps(line), flush=True)
    if check is not None and not check["ok"]:
        print(f"bench.py: the result check failed: {json.dumps(check)}", file=sys.stderr, flush=True)
        return 3
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
