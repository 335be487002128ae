#!/usr/bin/env python3
"""LDS bank model of the 1024-point wavefront FFT (csrc/thz_wfft.hpp): the float-image exchanges
(ds_write_b32 / ds_read_b32, 2 groups of 32 lanes, bank = dword mod 32) with the per-exchange
padding pad_s(j) = j + s (j >> 5), and the twiddle-table reads (ds_read_b64, bank = dword mod 64).
Prints the extra cycles per wave-instruction class for the round-2 layout and the round-3 one.
usage: wfft_bank_sim.py"""
import numpy as np

lane = np.arange(64)


def cyc(addr, mod):
    c = 0
    for g in (addr[:32], addr[32:]):
        banks = {}
        for a in set(int(x) for x in g):
            banks.setdefault(a % mod, set()).add(a)
        c += max(len(s) for s in banks.values())
    return c - 2  # extra cycles over a conflict-free access


def cyc64(idx):
    """ds_read_b64 of float2 entries idx: dwords 2 idx, 2 idx + 1, bank mod 64."""
    c = 0
    for g in (idx[:32], idx[32:]):
        banks = {}
        for e in set(int(x) for x in g):
            for d in (2 * e, 2 * e + 1):
                banks.setdefault(d % 64, set()).add(e)
        c += max(len(s) for s in banks.values())
    return c - 2


def exchanges(s1, s2):
    pad1 = lambda j: j + s1 * (j >> 5)
    pad2 = lambda j: j + s2 * (j >> 5)
    out = {}
    k1 = lane & 15
    out["fwd ex1 write"] = sum(cyc(pad1(16 * lane + q), 32) for q in range(16))
    out["fwd ex1 read"] = sum(cyc(pad1(lane + 64 * r), 32) for r in range(16))
    out["fwd ex2 write"] = sum(cyc(pad2((lane - k1) * 16 + k1 + 16 * q), 32) for q in range(16))
    out["fwd ex2 read"] = sum(cyc(pad2(lane + 64 * (b >> 2) + 256 * (b & 3)), 32) for b in range(16))
    k3 = lane & 3
    out["inv ex1 write"] = sum(cyc(pad1(4 * (lane + 64 * (a >> 2)) + (a & 3)), 32) for a in range(16))
    out["inv ex1 read"] = sum(cyc(pad1(lane + 64 * r), 32) for r in range(16))
    out["inv ex2 write"] = sum(cyc(pad2((lane - k3) * 16 + k3 + 4 * q), 32) for q in range(16))
    out["inv ex2 read"] = sum(cyc(pad2(lane + 64 * r), 32) for r in range(16))
    return out


def twiddles(new):
    out = {}
    k1 = lane & 15
    out["fwd st1 t256[16r+k]"] = sum(cyc64(16 * r + k1) for r in range(1, 16))
    f2 = 0
    for m in range(4):
        k = lane + 64 * m
        f2 += cyc64(k) + (cyc64(768 + k) if new else cyc64(2 * k)) + cyc64(3 * k)
    out["fwd st2 w^k, w^2k, w^3k"] = f2
    k3 = lane & 3
    out["inv st1 t64[k r]"] = sum(cyc64(k3 * r) for r in range(1, 16))
    out["inv st2 w^(lane r)"] = sum(cyc64(64 * (r - 1) + lane) if new else cyc64(lane * r) for r in range(1, 16))
    return out


for name, (s1, s2, new) in {"round 2": (1, 1, False), "round 3": (1, 2, True)}.items():
    ex, tw = exchanges(s1, s2), twiddles(new)
    print(f"{name}: exchanges {ex}\n         twiddles {tw}\n         total extra cycles per transform pair "
          f"{sum(ex.values()) + sum(tw.values())}")
