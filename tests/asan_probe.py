"""Deliberate heap overflow through the oracle's C code (run by
tests/test_sanitizers.py under the ASan build: proves the instrumentation is
live).  orc_set_state reads side*side ground bytes; it is handed 10."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle.oracle import OracleEnv, Params, lib  # noqa: E402

L = lib()
e = OracleEnv(Params(side=8, n_drones=2))
vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
g = np.zeros(10, np.uint8)  # malloc'd by numpy: ASan redzones around it
o, y, x = np.arange(2, dtype=np.int32), np.zeros(2, np.int32), np.arange(2, dtype=np.int32)
c, p = np.full(2, 100, np.int32), np.zeros(2, np.uint8)
L.orc_set_state(e._e, vp(g), vp(o), vp(y), vp(x), vp(c), vp(p), None)
print("no report")
