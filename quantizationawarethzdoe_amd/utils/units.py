"""Length/time unit constants (reference utils/units.py:1-11)."""
nm = 1 * 10 ** -9
um = 1 * 10 ** -6
mm = 1 * 10 ** -3
cm = 1 * 10 ** -2
m = 1

s = 1
ms = 1 * 10 ** -3
us = ms * 1 * 10 ** -3
ns = us * 1 * 10 ** -3
