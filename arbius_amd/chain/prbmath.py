"""Exact integer re-implementation of the PRBMath fixed-point functions EngineV1
uses (UD60x18 / SD59x18 ``exp2``, ``div``, ``mul``), so MockEngine reproduces
the contract's reward math bit-for-bit (goldens: contract/test/reward.test.ts:152-231).

``Common.exp2`` multiplies a 192.64 accumulator by sqrt-chain constants
2^(2^-k) in 64.64 (round-to-nearest; first eight checked against PRBMath's
literals) for every set fractional bit, then rescales to 18 decimals.
"""
from __future__ import annotations

from decimal import Decimal, getcontext

UNIT = 10 ** 18
_C = None


def _consts():
    global _C
    if _C is None:
        getcontext().prec = 100
        two = Decimal(2)
        out = {}
        for bit in range(64):
            v = (two ** (two ** (bit - 64))) * (two ** 64)
            out[bit] = int(v.to_integral_value())  # ROUND_HALF_EVEN; no ties occur
        _C = out
    return _C


def common_exp2(x_192x64: int) -> int:
    c = _consts()
    result = 1 << 191
    for bit in range(63, -1, -1):
        if x_192x64 & (1 << bit):
            result = (result * c[bit]) >> 64
    result *= UNIT
    result >>= (191 - (x_192x64 >> 64))
    return result


def ud_exp2(x: int) -> int:
    if x > 192 * UNIT - 1:
        raise OverflowError("PRBMath_UD60x18_Exp2_InputTooBig")
    return common_exp2((x << 64) // UNIT)


def ud_div(x: int, y: int) -> int:
    return (x * UNIT) // y


def _tdiv(a: int, b: int) -> int:
    """Solidity-style division truncating toward zero."""
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b >= 0) else -q


def sd_div(x: int, y: int) -> int:
    return _tdiv(x * UNIT, y)


def sd_mul(x: int, y: int) -> int:
    return _tdiv(x * y, UNIT)


def sd_exp2(x: int) -> int:
    if x < 0:
        if x < -59_794_705_707_972_522_261:
            return 0
        return _tdiv(UNIT * UNIT, sd_exp2(-x))
    if x > 192 * UNIT - 1:
        raise OverflowError("PRBMath_SD59x18_Exp2_InputTooBig")
    return common_exp2((x << 64) // UNIT)
