#!/usr/bin/env python3
"""max |a - b| per array of two tools/enc_dump.py outputs"""
import sys
import numpy as np
a, b = np.load(sys.argv[1]), np.load(sys.argv[2])
print({k: float(np.abs(a[k] - b[k]).max()) for k in a.files})
