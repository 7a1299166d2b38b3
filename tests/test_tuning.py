"""Kernel tuning knobs (csrc/runtime/tuning.h): one registry, validated values, settable in-process."""
import pytest


def test_set_knob_validates(native):
    from mipipe import _native as N
    L = N.lib()
    assert L.mp_set_knob(b"GEMVS_NS", 3) == 0
    assert L.mp_set_knob(b"GEMVS_NS", 2) == 0
    # NS 8 was silently run as NS 4 before: now refused
    assert L.mp_set_knob(b"GEMVS_NS", 8) != 0
    assert b"out of range" in L.mp_last_error()
    assert L.mp_set_knob(b"NO_SUCH_KNOB", 1) != 0
    assert b"unknown knob" in L.mp_last_error()
    assert L.mp_set_knob(b"GEMV_NW", 6) != 0
    assert L.mp_set_knob(b"GEMV_NW", 8) == 0
