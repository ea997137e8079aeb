"""bench.py's stdout line: the driver keeps only the tail of stdout, so the line is a compact summary
(< 4 KB) of the full record (written to --detail).  Built here from round 5's full record
(profiles/r05/v6_bench.json) with its 8-GPU shard leg recast as the 2/4/8 strong_split."""
import json
import os

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _full_line():
    with open(os.path.join(ROOT, "profiles", "r05", "v6_bench.json")) as f:
        line = json.load(f)
    leg = line.pop("strong_shard_8gpu")
    line["strong_split"] = {"2": dict(leg, gpus=2), "4": dict(leg, gpus=4), "8": leg}
    line["roofline"]["on_chip"] = bench.on_chip_roofline(line["roofline"]["amp_terms_per_launch"],
                                                         line["roofline"]["avg_launch_us"] * 1e-3, 17.0)
    return line


def test_compact_line_is_small_and_carries_the_contract():
    line = _full_line()
    c = bench.compact_line(line, "gpurun_out/bench_detail.json")
    s = json.dumps(c)
    assert len(s) < 4096, len(s)
    assert len(json.dumps(line)) > 3 * len(s)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in c, k
    assert c["value"] == line["value"]
    r = c["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in r, k
    assert r["kernel"] == "k_interval<13, true>"
    assert 0.0 < r["on_chip"]["lds_frac"] < 1.0
    assert c["cpu_baseline"]["kind"] == "port" and c["cpu_baseline"]["cores"] == 1
    fs = c["full_sweep"]
    assert abs(fs["value"] - line["full_sweep"]["value"]) < 1e-4 * fs["value"] and fs["engine"]
    assert fs["tolerance_at_t_final"]["value"] <= 1e-8
    assert set(c["strong_split"]) >= {"2", "4", "8"}
    assert abs(c["strong_split"]["8"]["step_ms"] - line["strong_split"]["8"]["step_ms"]) < 0.05
    assert "shards" not in json.dumps(c["strong_split"])
    assert c["large_register"]["kernel_ms_per_h_application"] > 0
    assert c["detail"] == "gpurun_out/bench_detail.json"


def test_lds_bytes_per_amp_term_matches_the_kernel_schedule():
    # 16 amplitudes per thread; per term 9 x (16 + 64 + 8) + 19 + 16 ds_read_b128 and 16 ds_write_b128
    assert bench.LDS_B_PER_AMP_TERM == 16.0 * (9 * 88 + 51) / 16.0
    assert abs(bench.LDS_PEAK_TBS - 157.3) < 0.1


def test_clock_under_load_record_is_read():
    """roofline.on_chip.clock: the GPU clock under the bench's full sweep from the committed
    GRBM_GUI_ACTIVE record (tools/clock_probe.sh), below the nominal 2.4 GHz and below the clock of
    one GPU's 2-GPU share (the chip power-caps with every CU busy)."""
    clk = bench.clock_under_load()
    assert clk is not None
    assert 1.0 < clk["full_sweep_ghz"] < clk["share2_ghz"] <= 2.4
