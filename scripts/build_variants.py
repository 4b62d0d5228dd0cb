"""Build tuning variants of the HIP library: python scripts/build_variants.py NAME K=V [K=V ...] ..."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from distributed_learning_simulation_lib_amd.build import LIB_DIR, build  # noqa: E402

args = sys.argv[1:]
name, defs = None, {}
variants = []
for a in args + ["--"]:
    if "=" in a:
        k, v = a.split("=", 1)
        defs[k] = int(v)
    else:
        if name is not None:
            variants.append((name, defs))
        name, defs = a, {}
for name, defs in variants:
    print(build(defines=defs, out=LIB_DIR / "variants" / f"lib_{name}.so"))
