"""Regenerates tests/golden/goal_rng.json: the goals JSBSimEnv.reset(seed) draws
(jsbsim_gym.py:312-323), restated with numpy's default_rng -- no reference code is run.
The SURVEY.md 8c vectors for seeds 0, 1, 42 are included and cross-checked by the test."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from f16_jsb_amd.env import reference_goal  # noqa: E402

if __name__ == "__main__":
    out = {"source": "jsbsim_gym/jsbsim_gym.py:312-323 restated with numpy %s default_rng (tests/golden/make_goal_rng.py)" % np.__version__,
           "goals": {str(s): reference_goal(s).tolist() for s in (0, 1, 2, 3, 7, 42, 123, 2**31 - 1)}}
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "goal_rng.json"), "w") as f:
        json.dump(out, f, indent=1)
