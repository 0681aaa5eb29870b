"""LAPF 3-source step 1, headless: the initial-guess file "xca yca xcb ycb xcc ycc bkgdx
bkgdy" from given positions of A, B, C and an empty sky patch (3body/apf_step1_3body.py
takes them from mouse clicks; see olpefit_amd/step1.py).

    python 3body/apf_step1_3body.py <directory> --star X Y --companion X Y --companion X Y --sky X Y
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from olpefit_amd.step1 import main  # noqa: E402

if __name__ == "__main__":
    main(three_body=True)
