"""Per-unit start/end times of one sampler launch (diagnostic library built with
-DOLPE_DIAG_SPAN, tools/diag_build.sh): how a launch's time splits into start-up,
steady running and the tail, and how evenly the waves of a SIMD progress.

    OLPE_LIB=diag/span/libolpe.so python tools/span_diag.py [walkers] [iters] [units]
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 3072
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    units = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    os.environ["OLPE_UNITS"] = str(units)
    from olpefit_amd import synth
    from olpefit_amd.core import Sampler
    from olpefit_amd.pipeline import initial_parameters
    img, _ = synth.make_image(64, 2, 0)
    p0 = initial_parameters(img, synth.guess_values(64, 2), 2)
    s = Sampler(img, 1.0, 1, 1, 2, nsrc=2)
    p0[-1] = s.chi_squared(p0)
    s.seed(1000 + np.arange(W))
    s.set_state(np.tile(p0, (W, 1)))
    s.enable_trace(True)
    # back to back, as bench.py queues them (no idle gap before the traced launch)
    for _ in range(int(os.environ.get("SPAN_LAUNCHES", "6"))):
        s.run_async(iters, burn_in=0, record_stride=10)
    s.sync()
    km = s.kernel_times(1)[0]
    P = s.last_units()
    tr = s.trace(iters).reshape(W, -1)[:, :5 * P].reshape(W, P, 5)
    t0, t1 = tr[..., 0] * 10e-6, tr[..., 1] * 10e-6          # ms
    base = t0.min()
    t0, t1 = t0 - base, t1 - base
    hw = tr[..., 2].astype(np.int64)
    xcc = tr[..., 3].astype(np.int64)
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 15
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    slot = ((xcc * 8 + se) * 2 + sh) * 16 + cu
    dur = t1 - t0
    clk = tr[..., 4] / (dur * 1e-3) / 1e9                  # s_memtime ticks per second (GHz)
    q = lambda a: " ".join(f"{np.percentile(a, p):.3f}" for p in (0, 10, 50, 90, 100))
    print(f"W={W} iters={iters} units={P} kernel_ms={km:.3f}  (percentiles 0/10/50/90/100)")
    print(f"  unit start ms: {q(t0)}")
    print(f"  unit end   ms: {q(t1)}")
    print(f"  unit dur   ms: {q(dur)}")
    print(f"  s_memtime rate GHz: {q(clk)}")
    print(f"  last end - kernel: {t1.max():.3f} of {km:.3f}")
    # spread of end times among the waves of one SIMD (last unit of each walker)
    key = slot * 4 + simd
    ends = {}
    for k, e in zip(key[:, -1], t1[:, -1]):
        ends.setdefault(int(k), []).append(e)
    spread = np.array([max(v) - min(v) for v in ends.values() if len(v) > 1])
    nper = np.array([len(v) for v in ends.values()])
    print(f"  SIMDs seen {len(ends)}, walkers per SIMD {q(nper)}; end spread within a SIMD ms: {q(spread)}")
    cu_ends = {}
    for k, e in zip(slot[:, -1], t1[:, -1]):
        cu_ends.setdefault(int(k), []).append(e)
    cspread = np.array([max(v) - min(v) for v in cu_ends.values()])
    print(f"  CUs seen {len(cu_ends)}; end spread within a CU ms: {q(cspread)}")
    print(f"  busy fraction of wave-slots: {dur.sum() / (3072 * km):.3f}")
    s.close()


if __name__ == "__main__":
    main()
