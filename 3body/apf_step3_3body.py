"""LAPF 3-source step 3 front end (3body/apf_step3_3body.py's arguments, read of the
20-column chains and Gelman-Rubin statistics; see olpefit_amd/step3.py).

    python 3body/apf_step3_3body.py <image> <system> -s <walkers> [-a <burn>]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from olpefit_amd.step3 import main  # noqa: E402

if __name__ == "__main__":
    main(nsrc=3)
