"""Debug: the mixed_dtypes golden case through the plugin: waves of 1, 3 (host updates), 64."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from tests.golden_io import bits_equal  # noqa: E402
from tests import test_gpu_parity as tp  # noqa: E402

dev = torch.device("cuda", 0)
case = tp.CASES["mixed_dtypes"]
for wave, host in ((1, False), (3, True), (64, False), (64, False)):
    algos = []
    res = tp.run_hip(case, dev, wave, from_host=host, algo_out=algos)
    bad = [k for k, want in case.expected.items() if not bits_equal(res.parameter[k].cpu().numpy(), want)]
    print("wave", wave, "host", host, "bad", bad, "stats", algos[0].dyn_stats, flush=True)
    for k in bad:
        g = res.parameter[k].cpu().numpy().ravel()
        for i, a in enumerate(case.arrivals):
            x = np.asarray(a.arrays[k], dtype=np.float64).ravel()
            print("  client", i, "equal raw:", np.array_equal(g, x), "close:", np.allclose(g, x))
        print("  got", g[:3], "want", case.expected[k].ravel()[:3])
