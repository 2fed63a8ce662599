"""Locate glibc's powf data tables in the system libm and print them as C++ hex-float
constants (rust_tracer_amd/csrc/rt_powf.hpp holds the output).

glibc >= 2.28 evaluates powf (sysdeps/ieee754/flt-32/e_powf.c, from ARM's optimized-routines)
in double with two tables: __powf_log2_data (16 {invc, logc} pairs + 5 polynomial
coefficients) and __exp2f_data (32 uint64 + scalars).  Both are hidden symbols, so they are
found by value: the exp2 table is tab[i] = asuint64(2^(i/32)) - (i << 47) (computable), the
log2 table is the run of 16 {invc, logc ~ -log2(invc)} pairs followed by 5 coefficients whose
last is ~1/ln 2.  The device's powf (rt_powf.hpp) replays glibc's algorithm with these
constants, so that specular terms are bit-identical to the reference's libm powf.
"""
import math
import struct
import sys
from decimal import Decimal, getcontext

getcontext().prec = 60
path = sys.argv[1] if len(sys.argv) > 1 else "/lib/x86_64-linux-gnu/libm.so.6"
data = open(path, "rb").read()
tab = []
for i in range(32):
    d = float(Decimal(2) ** (Decimal(i) / Decimal(32)))
    u = struct.unpack("<Q", struct.pack("<d", d))[0]
    tab.append((u - (i << 47)) & 0xFFFFFFFFFFFFFFFF)
pat = b"".join(struct.pack("<Q", t) for t in tab)
e = data.find(pat)
assert e >= 0 and data.find(pat, e + 1) < 0, "exp2f table not found exactly once"
shift_scaled, p0, p1, p2 = struct.unpack_from("<4d", data, e + 256)
assert shift_scaled == float.fromhex("0x1.8p+47")
log2 = None
for off in range(0, len(data) - 37 * 8, 8):
    v = struct.unpack_from("<37d", data, off)
    if all(0.6 < v[2 * i] < 1.6 and math.isfinite(v[2 * i + 1]) and abs(v[2 * i + 1] + math.log2(v[2 * i])) < 1e-9
           for i in range(16)) and abs(v[36] - 1 / math.log(2)) < 1e-6 and abs(v[35] + 0.5 / math.log(2)) < 1e-3:
        assert log2 is None, "log2 table ambiguous"
        log2 = v
assert log2 is not None, "powf log2 table not found"
print("// __powf_log2_data.tab {invc, logc}")
for i in range(16):
    print(f"    {{{log2[2 * i].hex()}, {log2[2 * i + 1].hex()}}},")
print("// __powf_log2_data.poly")
print("    " + ", ".join(x.hex() for x in log2[32:37]))
print("// __exp2f_data.tab")
for i in range(0, 32, 4):
    print("    " + ", ".join(f"0x{t:016x}ull" for t in tab[i:i + 4]) + ",")
print("// __exp2f_data.shift_scaled, poly")
print("    " + ", ".join(x.hex() for x in (shift_scaled, p0, p1, p2)))
