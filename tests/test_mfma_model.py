"""bench.py's issued matrix-cycle model (mfma_cycles, the numerator of every
`frac_issued`) against the SQ counters of the kernels it describes.

profiles/r05/final/mfma_c4.json is scripts/mfma_check.py's summary of an eager
C4 run under `rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA` on the
round-5 kernels: for each MFMA stage, the busy cycles the counter saw per
dispatch.  The model must reproduce them exactly (a kernel change that alters
its instruction count has to update bench.mfma_cycles, and this fixture is
re-measured with scripts/gpu_r5.sh mfma_c4)."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

FIXTURE = os.path.join(ROOT, "profiles", "r05", "final", "mfma_c4.json")


@pytest.mark.parametrize("stage", ["conv_fwd", "fc_fwd", "fc_bwd", "conv_bwd"])
def test_issued_cycle_model_equals_counter(stage):
    if not os.path.exists(FIXTURE):
        pytest.skip("no counter fixture")
    d = json.load(open(FIXTURE))[stage]
    arch, n, _ = bench.WORKLOADS["c4"]
    model = bench.mfma_cycles(stage, n, 5, arch)
    assert model == d["model_cycles"]
    assert model == d["busy_cycles"], (stage, model, d["busy_cycles"])
    # 16 cycles per bf16 16x16x32 and 32 per f32 16x16x4: the instruction count bounds the cycles
    assert 16 * d["mfma_insts"] <= d["busy_cycles"] <= 32 * d["mfma_insts"]


def test_ideal_cycles_never_exceed_issued():
    """padding = issued / ideal >= 1 for every MFMA stage of both nets (the
    ideal counts the algorithmic FLOPs at the same instruction rates)."""
    for stage in ("conv_fwd", "fc_fwd", "fc_bwd", "conv_bwd"):
        for n in (75, 256, 512, 1024):
            assert bench.mfma_cycles(stage, n, 5, "ff") >= 0.999 * bench.mfma_ideal_cycles(stage, n, 5), (stage, n)
    for stage in ("lstm_gates", "lstm_bptt"):
        for n in (80, 512, 1024):
            assert bench.mfma_cycles(stage, n, 5, "lstm") >= 0.999 * bench.mfma_ideal_cycles(stage, n, 5), (stage, n)
