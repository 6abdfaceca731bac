"""bench.py's output contract on a real GPU, at a small size: the driver parses exactly ONE JSON line
from stdout (native libraries' banners must not reach it), with the metric / value / unit / roofline
/ cpu_baseline fields the contract names, for the single-GPU step and the forced exchange path
(the N > 1 code path at world 1, whose RCCL initialisation prints a version banner)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--points", "20000", "--width", "320", "--height", "240", "--views", "16", "--steps", "3", "--warmup", "2",
         "--sync-loss-steps", "2", "--fwd-frames", "2", "--no-cpu-baseline"]


def _run(args):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       timeout=280, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.parametrize("extra", [[], ["--force-dist"]])
def test_bench_prints_one_json_line(extra):
    # started before this process touches the GPU (conftest.py runs this module first; no `gpu`
    # fixture here: torch.cuda.is_available() would initialise it, device_count() does not)
    import torch

    if torch.cuda.device_count() == 0:
        pytest.skip("no HIP device")
    line = _run(SMALL + extra)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in line, k
    assert line["n_gpus"] == 1 and line["steps"] == 3 and line["warmup"] == 2
    assert line["value"] > 0 and line["ms_per_step"] > 0
    assert abs(line["value"] * line["ms_per_step"] - 1000.0) < 0.05 * 1000.0
    assert line["roofline"]["unit"] == "GB/s" and line["roofline"]["achieved"] > 0
    assert ("RCCL" in line["config"]["parallelism"]) == bool(extra)
