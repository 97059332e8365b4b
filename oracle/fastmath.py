"""Bit-exact restatement of the reference's scalar fast-math helpers (test infrastructure).

The vMF loss and the lbessel op use P. Mineiro's bit-trick approximations, which differ
from libm by large constants.  They are scalar functions of constants of the
problem (D, nu), so the engine evaluates them on the host; these numpy versions are the
oracle, pinned against the reference's own headers compiled into ``oracle/_ref``.
"""
import numpy as np


def fasterlog(x):
    """``fasterlog`` — reference ``include/utils/fastlog.h:75-85``.

    Reinterpret the float's bits as uint32, convert that integer to float32, scale by
    8.2629582881927490e-8f and subtract 87.989971088f (all in float32).
    """
    xf = np.asarray(x, dtype=np.float32)
    i = xf.view(np.uint32)
    y = i.astype(np.float32)
    y = y * np.float32(8.2629582881927490e-8)
    return np.float32(y - np.float32(87.989971088))


def fasterlgamma(x):
    """``fasterlgamma`` — reference ``include/utils/fastgamma.h:58-60``.

    -0.0810614667f - x - fasterlog(x) + (0.5f + x) * fasterlog(1.0f + x), float32 throughout.
    """
    x = np.float32(x)
    a = np.float32(np.float32(-0.0810614667) - x)
    a = np.float32(a - fasterlog(x))
    b = np.float32(np.float32(0.5) + x) * fasterlog(np.float32(np.float32(1.0) + x))
    return np.float32(a + np.float32(b))
