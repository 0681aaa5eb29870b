"""LAPF step 2a on MI355X: the optional single-walker warm-up (reference apf_step2a.py,
n_steps = 5000) writing <frame>_apf_results/step2a.csv, which ``apf_step2.py -i 2a``
starts from.  The reference's script fails as shipped (undefined ``burn_in`` at
apf_step2a.py:310); here burn-in defaults to 0."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from olpefit_amd.step2 import main  # noqa: E402

if __name__ == "__main__":
    main(nsrc=2, variant="2a")
