"""Test-side re-export of the repo's synthetic workload model."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from firedancer_amd.workload import (c2_mutate, L_INT, P_INT, SMALL_ORDER_ENCODINGS,  # noqa: E402,F401
                                     KIND_VALID)
