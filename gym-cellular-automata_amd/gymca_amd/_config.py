"""dtype policy mirrored from the reference (_config.py:11-12)."""
import numpy as np

TYPE_BOX = np.float64
TYPE_INT = np.int64
