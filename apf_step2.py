"""LAPF step 2 on MI355X -- drop-in for the reference's apf_step2.py entry point.

    python apf_step2.py <dir>/N2.<date>.<frame>.LDIF.fits [-i 1|2a] [--walkers W] ...

Same positional image, ``-i`` option, output directory and chain/acceptance files as
the reference (apf_step2.py:154-173, :342-365); the Gibbs/MH loop runs as a fused HIP
kernel on the GPU (olpefit_amd).  See ``--help`` for the added flags.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from olpefit_amd.step2 import main  # noqa: E402

if __name__ == "__main__":
    main(nsrc=2)
