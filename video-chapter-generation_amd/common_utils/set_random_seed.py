"""Seed every RNG the drivers use (`common_utils/set_random_seed.py:6-10` fixes 123 everywhere)."""
import random

import numpy as np
import torch


def use_fix_random_seed(seed=123):
    np.random.seed(seed)
    random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)
