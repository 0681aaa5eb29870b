"""Round 6 probe: where a 2-rank olpe_comm_init whose rank 1 never arrives spends its
time (non-blocking RCCL set-up, then the abort).  Prints each stage with a timestamp."""
import faulthandler
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
from olpefit_amd import synth
from olpefit_amd.core import Sampler
from olpefit_amd._lib import OlpeError

faulthandler.dump_traceback_later(40, exit=True)
t0 = time.time()


def say(*a):
    print(f"[{time.time() - t0:6.2f}s]", *a, flush=True)


img, _ = synth.make_image(32, 2, 0)
s = Sampler(img, 1.0, 1, 1, 2, nsrc=2)
s.seed(np.arange(4))
s.set_state(np.tile(np.arange(17, dtype=float) + 1.0, (4, 1)))
s.comm_timeout(float(sys.argv[1]) if len(sys.argv) > 1 else 4.0)
say("comm_init 2 ranks, rank 1 absent")
try:
    s.comm_init(Sampler.comm_unique_id(), 2, 0)
    say("JOINED")
except OlpeError as e:
    say("ERR", e.code, str(e)[:300])
s.nranks = 2
try:
    s.allgather_state()
except OlpeError as e:
    say("AFTER", e.code)
s.comm_timeout(600)
s.comm_init(Sampler.comm_unique_id(), 1, 0)
say("REJOIN", s.comm_info(), s.allgather_state().shape)
s.close()
say("closed")
