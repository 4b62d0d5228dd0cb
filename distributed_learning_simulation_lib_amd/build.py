"""Build the gfx950 HIP library in-tree (``_lib/libfedavg_hip.so``).

The library is the C-ABI declared in ``include/fedavg_hip.h``. It is compiled with
``hipcc --offload-arch=gfx950`` straight from ``csrc/`` — no torch extension machinery, no
JIT cache: the built ``.so`` lives next to the package so it travels with the repository
snapshot to the GPU box.
"""

from __future__ import annotations

import os
import shutil
import subprocess
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
REPO_DIR = PKG_DIR.parent
CSRC = PKG_DIR / "csrc"
LIB_DIR = PKG_DIR / "_lib"
LIB_NAME = "libfedavg_hip.so"
LIB_PATH = LIB_DIR / LIB_NAME
SOURCES = [CSRC / "fedavg_kernels.hip", CSRC / "personalized_kernels.hip", CSRC / "host_pack.cpp",
           CSRC / "sharded_comm.cpp", CSRC / "multi_device.cpp"]
HEADERS = [REPO_DIR / "include" / "fedavg_hip.h", CSRC / "exact_div.h", CSRC / "rccl_bind.h"]
# C++ clients of the ABI alone (no Python, no torch), built next to the library
EXAMPLES = {"c_abi_round": REPO_DIR / "examples" / "c_abi_round.cpp",
            "multi_device_round": REPO_DIR / "examples" / "multi_device_round.cpp",
            # test infrastructure: the native multi-rank round with ranks as threads on one GPU
            "threaded_ranks": REPO_DIR / "tests" / "native" / "threaded_ranks.cpp"}
# test infrastructure: in-process RCCL stand-ins for threaded_ranks (tests/native/fake_rccl.cpp),
# with ncclGather and without it (the grouped send / recv fallback of sharded_comm.cpp)
FAKE_RCCL_SRC = REPO_DIR / "tests" / "native" / "fake_rccl.cpp"
FAKE_RCCL = {"libfake_rccl.so": [], "libfake_rccl_nogather.so": ["-DFAKE_RCCL_NO_GATHER"]}
# host-side staging of plugin updates: a torch C++ extension (CPU code; the C ABI above stays
# torch-free), built in-tree into _lib/staging/ so it travels with the snapshot
STAGING_SRC = CSRC / "staging_ext.cpp"
STAGING_NAME = "fedavg_staging"
STAGING_DIR = LIB_DIR / "staging"
STAGING_PATH = STAGING_DIR / f"{STAGING_NAME}.so"

# -ffp-contract=off: the reference rounds the fp64 product and the fp64 sum separately
# (torch `x.to(f64) * w` then `acc += tmp`); an FMA would change low bits.
HIPCC_FLAGS = [
    "--offload-arch=gfx950",
    "-O3",
    "-std=c++17",
    "-ffp-contract=off",
    "-fPIC",
    "-shared",
    "-Wall",
    "-Wno-unused-function",
]


def hipcc() -> str:
    cand = os.environ.get("HIPCC") or shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    return cand


def needs_build() -> bool:
    if not LIB_PATH.exists():
        return True
    mtime = LIB_PATH.stat().st_mtime
    return any(p.stat().st_mtime > mtime for p in SOURCES + HEADERS + [Path(__file__)])


def build(force: bool = False, verbose: bool = False, defines: dict[str, int] | None = None,
          out: Path | None = None) -> Path:
    """Compile the HIP library for gfx950. Returns the path of the shared object.

    ``defines``/``out`` build a tuning variant (e.g. ``{"FEDAVG_NT": 1}``) to another path.
    """
    target = out or LIB_PATH
    if out is None and not defines and not force and not needs_build():
        build_examples(verbose=verbose)
        build_staging(verbose=verbose)
        return LIB_PATH
    target.parent.mkdir(parents=True, exist_ok=True)
    tmp = target.with_suffix(".so.tmp")
    dflags = [f"-D{k}={v}" for k, v in (defines or {}).items()]
    cmd = [hipcc(), *HIPCC_FLAGS, *dflags, f"-I{REPO_DIR / 'include'}", *map(str, SOURCES), "-o", str(tmp)]
    if verbose:
        print(" ".join(cmd))
    proc = subprocess.run(cmd, capture_output=True, text=True)
    if proc.returncode != 0:
        raise RuntimeError(f"hipcc failed ({proc.returncode}):\n{proc.stdout}\n{proc.stderr}")
    os.replace(tmp, target)
    if out is None:
        build_examples(verbose=verbose)
        build_staging(verbose=verbose)
    return target


def build_staging(force: bool = False, verbose: bool = False) -> Path | None:
    """Compile the staging extension (torch.utils.cpp_extension, g++) into _lib/staging/. It is an
    accelerator of the plugin's host staging, so a failed build warns instead of failing the
    library build (the plugin then stages in Python)."""
    try:
        return _build_staging(force, verbose)
    except Exception as e:  # noqa: BLE001 - optional component
        print(f"warning: staging extension not built ({e}); the plugin will stage updates in Python")
        return None


def _build_staging(force: bool, verbose: bool) -> Path:
    if not force and STAGING_PATH.exists() and STAGING_PATH.stat().st_mtime > STAGING_SRC.stat().st_mtime:
        return STAGING_PATH
    from torch.utils import cpp_extension

    STAGING_DIR.mkdir(parents=True, exist_ok=True)
    cpp_extension.load(name=STAGING_NAME, sources=[str(STAGING_SRC)], build_directory=str(STAGING_DIR),
                       extra_cflags=["-O3"], verbose=verbose)
    return STAGING_PATH


def _run(cmd: list[str], what: str, verbose: bool) -> None:
    if verbose:
        print(" ".join(cmd))
    proc = subprocess.run(cmd, capture_output=True, text=True)
    if proc.returncode != 0:
        raise RuntimeError(f"hipcc failed for {what} ({proc.returncode}):\n{proc.stdout}\n{proc.stderr}")


def build_examples(verbose: bool = False) -> list[Path]:
    """Link each example against the in-tree library (rpath $ORIGIN: they live in _lib/), and
    build the test-only RCCL stand-ins."""
    built = []
    for name, extra in FAKE_RCCL.items():
        so = LIB_DIR / name
        if not (so.exists() and so.stat().st_mtime > FAKE_RCCL_SRC.stat().st_mtime):
            _run([hipcc(), "-O2", "-std=c++17", "-fPIC", "-shared", *extra, str(FAKE_RCCL_SRC), "-o", str(so)],
                 FAKE_RCCL_SRC.name, verbose)
        built.append(so)
    for name, src in EXAMPLES.items():
        exe = LIB_DIR / name
        if exe.exists() and exe.stat().st_mtime > max(src.stat().st_mtime, LIB_PATH.stat().st_mtime):
            built.append(exe)
            continue
        _run([hipcc(), "--offload-arch=gfx950", "-O2", "-std=c++17", "-ffp-contract=off", f"-I{REPO_DIR / 'include'}",
              str(src),
              f"-L{LIB_DIR}", "-lfedavg_hip", "-pthread", "-Wl,-rpath,$ORIGIN", "-o", str(exe)], src.name, verbose)
        built.append(exe)
    return built


if __name__ == "__main__":
    print(build(force=True, verbose=True))
