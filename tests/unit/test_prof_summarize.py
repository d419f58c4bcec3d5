"""tools/prof_summarize.py: the timed window of a bench trace is the first window between two idle
gaps that the GPU kept busy (bench.py EWDML_PROF_GAP=1 sleeps before and after each timed loop; the
extra measurements and teardown after it add windows of their own), else the busiest, and the
report's per-step numbers come from that window only."""
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
    assert "90 % busy" in first and "40 kernels" in first
    assert "k_step" in txt and "k_warm" not in txt and "copyBuffer" not in txt
    assert "last step, 10 kernels" in txt


def test_headline_window_before_the_extra_measurements():
    warm, t = _kernels(0, 30, 10, "k_warm")
    head, t = _kernels(t + 250 * MS, 40, 20, "k_head_step")
    # an extra measurement: an eager setup window (more kernels, mostly idle), then its own
    # timed window (more kernels than the headline's)
    setup, t = _kernels(t + 250 * MS, 90, 5, "k_setup", gap_us=60)
    extra, t = _kernels(t + 250 * MS, 60, 20, "k_extra_step")
    end, _ = _kernels(t + 250 * MS, 2, 5, "k_end")
    txt = summarize(warm + head + setup + extra + end, steps=4)
    assert "40 kernels" in txt.splitlines()[0]
    assert "k_head_step" in txt and "k_extra_step" not in txt and "k_setup" not in txt


def test_busiest_window_when_none_is_dense():
    a, t = _kernels(0, 5, 10, "a")
    b, t = _kernels(t + 200 * MS, 30, 5, "b", gap_us=20)
    c, t = _kernels(t + 200 * MS, 12, 5, "c", gap_us=20)
    d, _ = _kernels(t + 200 * MS, 2, 5, "d")
    first = summarize(a + b + c + d).splitlines()[0]
    assert "busiest" in first and "30 kernels" in first


def test_single_gap_and_no_gap():
    a, t = _kernels(0, 5, 10, "a")
    b, _ = _kernels(t + 200 * MS, 6, 10, "b")
    assert "after last idle gap, 6 kernels" in summarize(a + b)
    c, _ = _kernels(0, 10, 10, "c")
    assert "last 50% of trace" in summarize(c)


def test_short_names_keep_template_arguments():
    assert short("void (anonymous namespace)::k_cf_gemm<0, 128, 128>(float const*, int)") == \
        "k_cf_gemm<0, 128, 128>"
