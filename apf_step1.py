"""LAPF step 1, headless: the initial-guess file from given click positions (the
reference's apf_step1.py takes them from mouse clicks).

    python apf_step1.py <directory> --star X Y --companion X Y --sky X Y
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from olpefit_amd.step1 import main  # noqa: E402

if __name__ == "__main__":
    main()
