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
