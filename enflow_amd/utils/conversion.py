"""Unit conversions to/from LJ units (mirrors enflow/utils/conversion.py:1-62).

Behaviour is kept identical to the reference, including that 'femto' uses the
pico factor in vel_to_lj / lj_to_vel (conversion.py:32-36, 55-59).
"""
import math

from .constants import M, sigma, eps, kB


def meter_to_lj(x):
    return x / sigma


def meter_per_sec_to_lj(x):
    return x * math.sqrt(M / eps)


def amu_to_lj(m):
    return m / M


def second_to_lj(t):
    return t * math.sqrt(eps / M) / sigma


def time_to_lj(t, unit='pico'):
    a = 1e-12 if unit == 'pico' else 1e-15
    return second_to_lj(t * a)


def dist_to_lj(x, unit='ang'):
    a = 1e-10 if unit == 'ang' else 1e-9
    return meter_to_lj(x * a)


def vel_to_lj(x, unit1='ang', unit2='pico'):
    a = 1e-10 if unit1 == 'ang' else 1e-9
    b = 1e-12
    return meter_per_sec_to_lj(x * a / b)


def kelvin_to_lj(T):
    return T * kB / eps


def lj_to_kelvin(kBT):
    return kBT * eps / kB


def lj_to_meter(x_):
    return x_ * sigma


def lj_to_meter_per_sec(x):
    return x * math.sqrt(eps / M)


def lj_to_dist(x_, unit='ang'):
    a = 1e-10 if unit == 'ang' else 1e-9
    return lj_to_meter(x_ / a)


def lj_to_vel(x_, unit1='ang', unit2='pico'):
    a = 1e-10 if unit1 == 'ang' else 1e-9
    b = 1e-12
    return lj_to_meter_per_sec(x_ * b / a)
