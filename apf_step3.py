"""LAPF step 3 front end on MI355X output -- the reference apf_step3.py's arguments, chain
read, burn-in and Gelman-Rubin statistics (its distortion / refraction stages need data
the reference does not ship; see olpefit_amd/step3.py).

    python apf_step3.py <dir>/N2.<date>.<frame>.LDIF.fits <system> -s <walkers> [-a <burn>]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from olpefit_amd.step3 import main  # noqa: E402

if __name__ == "__main__":
    main(nsrc=2)
