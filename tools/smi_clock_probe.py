"""Exploration (round 5): can the bench read the clock the GPU holds under the sampler's
load from the SMU, through ROCm's amdsmi package, without touching the GPU's queues?
Prints the metric keys once, then samples the GFX clock every 20 ms from a host thread
while sampler launches run (configs[2] shape), and after them."""
import os
import sys
import threading
import time

sys.path.insert(0, "/opt/rocm/share/amd_smi")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import amdsmi  # noqa: E402

amdsmi.amdsmi_init()
hs = amdsmi.amdsmi_get_processor_handles()
print("handles", len(hs), [amdsmi.amdsmi_get_gpu_device_bdf(h) for h in hs])
h = hs[0]
for name, fn in [("clock", lambda: amdsmi.amdsmi_get_clock_info(h, amdsmi.AmdSmiClkType.GFX)),
                 ("metrics", lambda: amdsmi.amdsmi_get_gpu_metrics_info(h))]:
    try:
        v = fn()
        if isinstance(v, dict):
            print(name, {k: v[k] for k in v if "clk" in k.lower() or "clock" in k.lower()
                         or "power" in k.lower() or "freq" in k.lower()})
        else:
            print(name, v)
    except Exception as e:  # noqa: BLE001
        print(name, "failed:", type(e).__name__, e)

from olpefit_amd import synth  # noqa: E402
from olpefit_amd.core import Sampler  # noqa: E402
from olpefit_amd.pipeline import initial_parameters  # noqa: E402

img, _ = synth.make_image(64, 2, 0)
s = Sampler(img, 1.0, 1, 1, 2, nsrc=2, device=0)
p0 = initial_parameters(img, synth.guess_values(64, 2), 2)
p0[-1] = s.chi_squared(p0)
W = 65536
s.seed(1000 + np.arange(W))
s.set_state(np.tile(p0, (W, 1)))
samples, stop = [], threading.Event()


def sample():
    while not stop.is_set():
        t = time.perf_counter()
        try:
            c = amdsmi.amdsmi_get_clock_info(h, amdsmi.AmdSmiClkType.GFX)
            m = amdsmi.amdsmi_get_gpu_metrics_info(h)
            samples.append((t, c.get("clk"), m.get("average_gfxclk_frequency"),
                            m.get("current_gfxclk"), m.get("average_socket_power")))
        except Exception as e:  # noqa: BLE001
            samples.append((t, "err", str(e)))
        time.sleep(0.02)


for _ in range(5):
    s.run_async(100, record_stride=10)
s.sync()
th = threading.Thread(target=sample, daemon=True)
th.start()
t0 = time.perf_counter()
for _ in range(100):
    s.run_async(100, record_stride=10)
s.sync()
t1 = time.perf_counter()
time.sleep(0.3)
stop.set()
th.join()
print(f"launches {t0:.3f}..{t1:.3f} ({(t1 - t0) * 10:.2f} ms per launch)")
for x in samples:
    print(f"{x[0] - t0:+.3f}", *x[1:])
