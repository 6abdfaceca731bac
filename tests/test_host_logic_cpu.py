"""Host-side logic with no device: the sharded step's row blocks and record-exchange chunking
(rain_amd/sharded.py) and bench.py's algorithmic-byte model of the per-Gaussian backward."""
import importlib.util
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


@pytest.mark.parametrize("P,world", [(1, 1), (255, 2), (20000, 3), (1_000_000, 8), (2_000_000, 4), (5_000_000, 8)])
def test_row_blocks_cover_every_row(P, world):
    from rain_amd.sharded import row_blocks

    Q, P_pad = row_blocks(P, world)
    assert Q % 256 == 0 and Q >= 256 and P_pad == world * Q and P_pad >= P
    assert (world - 1) * Q < P or Q == 256  # no rank is left with only padding unless P is tiny


@pytest.mark.parametrize("world,Q", [(1, 1_000_192), (2, 500_224), (4, 250_112), (8, 125_184), (8, 625_152),
                                     (2, 2_500_096)])
def test_record_chunks_tile_the_row_block(world, Q):
    from rain_amd.sharded import ShardedStep

    s = ShardedStep(None, 0, world)
    CR = s.chunk_rows(Q)
    assert CR % 256 == 0 or CR == Q
    n = -(-Q // CR)
    assert 1 <= n <= 4
    if world == 1 or Q < 2 * ShardedStep.FILL_ROWS:
        assert n == 1  # nothing to overlap, or chunks would under-fill the GPU
    else:
        assert n >= 2 and min(CR, Q - (n - 1) * CR) > 0
    s.rec_chunk_rows = 300  # the tests' override rounds down to a multiple of 256
    assert s.chunk_rows(Q) == 256


def test_gauss_bwd_byte_models():
    b = _bench()
    P, V, K, M = 1_000_000, 683_000, 16, 16
    single = b.gauss_bwd_bytes(P, V, K, M)
    # fused Adam: the 64-B accumulator line, (param, exp_avg, exp_avg_sq) read + written for 59
    # floats per Gaussian, the statistics of the visible ones
    assert single == 64 * P + 24 * 59 * P + 24 * V
    # the owner kernel at N ranks: 1/N of the Adam rows, one 40-B record per row and view
    for world in (2, 4, 8):
        rows = -(-P // world)
        assert b.gauss_bwd_views_bytes(P, K, M, world) == rows * (24 * 59 + 24) + 40 * rows * world
    st = {"num_visible": V, "l_eff": 847_636, "tiles": 8160, "num_binned": 2_287_356}
    assert b.algorithmic_bytes("gauss_bwd", st, P, 1920, 1080, K) == single
    assert b.algorithmic_bytes("gauss_bwd", st, P, 1920, 1080, K, 1, True) == b.gauss_bwd_views_bytes(P, K, M, 1)
    assert b.algorithmic_bytes("gauss_bwd", st, P, 1920, 1080, K, 8) == b.gauss_bwd_views_bytes(P, K, M, 8)


@pytest.mark.parametrize("gpus,env,plan", [
    (None, {}, ("run", 1)),                         # the driver's default: one rank, this process
    (1, {}, ("run", 1)),
    (8, {}, ("spawn", 8)),                          # `bench.py --gpus 8` with no launcher: spawn 8 ranks
    (2, {"WORLD_SIZE": "2"}, ("run", 2)),           # under torch.distributed.run
    (None, {"WORLD_SIZE": "4"}, ("run", 4)),
])
def test_bench_launch_plan(gpus, env, plan):
    assert _bench().launch_plan(gpus, env) == plan


def test_bench_launch_plan_forced_exchange():
    """--force-dist (the Gaussian-sharded step at world 1) needs a launcher's environment for its
    process group: without one it spawns one rank; under a launcher it runs in place."""
    b = _bench()
    assert b.launch_plan(1, {}, force_dist=True) == ("spawn", 1)
    assert b.launch_plan(None, {}, force_dist=True) == ("spawn", 1)
    assert b.launch_plan(1, {"WORLD_SIZE": "1", "RANK": "0"}, force_dist=True) == ("run", 1)


@pytest.mark.parametrize("gpus,env", [(4, {"WORLD_SIZE": "2"}), (1, {"WORLD_SIZE": "8"}), (0, {}),
                                      (2, {"WORLD_SIZE": "x"})])
def test_bench_launch_plan_refuses(gpus, env):
    what, msg = _bench().launch_plan(gpus, env)
    assert what == "error" and msg


def test_bench_refuses_gpus_world_mismatch_before_torch():
    """A launcher's WORLD_SIZE that differs from --gpus ends bench.py with a non-zero code, before
    torch is imported (so nothing has touched a GPU)."""
    import subprocess
    import sys

    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "-X", "importtime", os.path.join(ROOT, "bench.py"), "--gpus", "4"],
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 2
    assert "does not match WORLD_SIZE=2" in r.stderr
    assert " torch" not in "\n".join(l for l in r.stderr.splitlines() if "import time" in l)


def test_bench_spawn_runs_n_ranks(tmp_path):
    """--gpus N without a launcher: torch.distributed.run starts N ranks as a child process whose
    rank 0 prints the line, and the child's exit code is returned (a stub stands in for bench.py)."""
    import subprocess
    import sys

    stub = tmp_path / "stub.py"
    stub.write_text(
        "import json, os, sys\n"
        "if os.environ['RANK'] == '0':\n"
        "    print(json.dumps({'world': int(os.environ['WORLD_SIZE']), 'argv': sys.argv[1:],\n"
        "                      'addr': os.environ['MASTER_ADDR']}), flush=True)\n"
        "sys.exit(int(sys.argv[-1]))\n")
    b = _bench()
    cmd = b.spawn_command(3, ["--gpus", "3", "0"], 29555, str(stub))
    assert cmd[1:3] == ["-m", "torch.distributed.run"] and "--nproc-per-node=3" in cmd
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    code = ("import importlib.util, sys\n"
            f"spec = importlib.util.spec_from_file_location('b', {os.path.join(ROOT, 'bench.py')!r})\n"
            "m = importlib.util.module_from_spec(spec); spec.loader.exec_module(m)\n"
            f"sys.exit(m._spawn(3, ['--gpus', '3', sys.argv[1]], {str(stub)!r}))\n")
    r = subprocess.run([sys.executable, "-c", code, "0"], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1 and '"world": 3' in lines[0] and '"addr": "127.0.0.1"' in lines[0]
    r = subprocess.run([sys.executable, "-c", code, "3"], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
