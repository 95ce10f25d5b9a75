"""CPU: bench.py's host-side helpers -- the committed PMC summaries it scales `roofline.traffic`
and the effective clock from (the full-batch forward at N = 1, the row-split shard kernel of
the N = 8 strong-scaling line, the f32 forward)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def test_pmc_summaries_per_kernel():
    full = bench.load_pmc(True)
    shard = bench.load_pmc(True, row_split=True)
    f32 = bench.load_pmc(False)
    assert full and shard and f32
    # HBM bytes per decoded element: the f64 delta rows (16 N B) plus a little read traffic,
    # about the same per element whatever the batch
    for d in (full, shard):
        assert 16 * 256 * 0.45 < d["per_elem"] < 16 * 256 * 0.55, d
    assert abs(shard["per_elem"] / full["per_elem"] - 1) < 0.02
    assert "rs_8192" in shard["source"] and "rs_8192" not in full["source"]
    assert 2.0 < full["clock_ghz"] < 2.5 and 2.0 < shard["clock_ghz"] < 2.5
    assert f32["per_elem"] < full["per_elem"]
