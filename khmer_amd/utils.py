"""Table-sizing helpers (khmer/_oxli/utils.pyx:12-17 over
include/oxli/hashtable.hh:79-123), computed by libkhmer_hip.so."""
import ctypes

from ._lib import lib, check


def get_n_primes_near_x(n_primes, x):
    """The n largest primes strictly below x (x == 1 gives [1])."""
    n = int(n_primes)
    out = (ctypes.c_uint64 * max(n, 1))()
    found = ctypes.c_uint32()
    check(lib.kh_get_n_primes_near_x(n, int(x), out, ctypes.byref(found)))
    if found.value != n:
        raise RuntimeError("unable to find %d prime numbers < %d" % (n, int(x)))
    return [int(v) for v in out[:n]]


def is_prime(n):
    out = ctypes.c_int()
    check(lib.kh_is_prime(int(n), ctypes.byref(out)))
    return bool(out.value)
