"""LAPF step 2, three-source variant, on MI355X -- drop-in for the reference's
3body/apf_step2_3body.py (19 parameters + chi^2, burn_in 0, no -i option)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from olpefit_amd.step2 import main  # noqa: E402

if __name__ == "__main__":
    main(nsrc=3)
