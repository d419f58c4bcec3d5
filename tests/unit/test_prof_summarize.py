"""tools/prof_summarize.py: the timed window of a bench trace is the busiest window between two
idle gaps (bench.py EWDML_PROF_GAP=1 sleeps before and after the timed loop; teardown after it can
add idle gaps of its own), and the report's per-step numbers come from that window only."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))

from tools.prof_summarize import short, summarize  # noqa: E402

MS = 1_000_000  # ns


def _kernels(t0, n, dur_us, name, gap_us=1):
    rows, t = [], t0
    for _ in range(n):
        rows.append((t, t + dur_us * 1000, name))
        t += (dur_us + gap_us) * 1000
    return rows, t


def test_busiest_window_between_gaps():
    warm, t = _kernels(0, 30, 10, "void (anonymous namespace)::k_warm<1>(float*)")
    timed, t = _kernels(t + 250 * MS, 40, 20, "void (anonymous namespace)::k_step(int)")
    tail, t = _kernels(t + 250 * MS, 3, 5, "__amd_rocclr_copyBuffer")
    late, _ = _kernels(t + 300 * MS, 2, 5, "k_late")
    txt = summarize(warm + timed + tail + late, steps=4)
    first = txt.splitlines()[0]
    assert "busiest" in first and "40 kernels" in first
    assert "k_step" in txt and "k_warm" not in txt and "copyBuffer" not in txt
    assert "last step, 10 kernels" in txt


def test_single_gap_and_no_gap():
    a, t = _kernels(0, 5, 10, "a")
    b, _ = _kernels(t + 200 * MS, 6, 10, "b")
    assert "after last idle gap, 6 kernels" in summarize(a + b)
    c, _ = _kernels(0, 10, 10, "c")
    assert "last 50% of trace" in summarize(c)


def test_short_names_keep_template_arguments():
    assert short("void (anonymous namespace)::k_cf_gemm<0, 128, 128>(float const*, int)") == \
        "k_cf_gemm<0, 128, 128>"
