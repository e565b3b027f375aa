#!/usr/bin/env python3
"""Generate fe25519_asm.h: GF(2^255-19) arithmetic on 8x32-bit limbs for gfx950.

Why asm: hipcc lowers a C++ product-scanning multiply to ~250 VALU ops per
field multiply (64 v_mad_u64_u32 plus v_lshl_add_u64 / v_cmp / v_cndmask per
carry); written directly it is 64+8 v_mad_u64_u32 + 57 v_addc_co_u32 plus a
few moves.  On gfx950 v_mad_u64_u32, v_addc_co_u32 and the other VOP3
integer ops issue at ~4 cycles per wave64 instruction while v_mov / v_and /
v_lshrrev / v_add_u32 issue at ~2.5 (profiles/r01_valu_rates_*.txt), so the
multiply is built from the former and the bookkeeping from the latter.

Representation: a field element is 8 little-endian u32 limbs holding any
value in [0, 2^256) ("loose").  "Tight" means < 2^255 + 2^43.
  fe_mul(r, a, b): loose x loose -> tight
  fe_add(r, a, b): loose + loose -> tight
  fe_sub(r, a, b): loose - tight -> loose     (b must be tight)

Multiply schedule (product scanning, "high columns first"):
  1. columns 8..14 of a*b (28 products) -> H = h0..h7 (the top 256 bits of
     the product, minus the carry out of the low columns);
  2. columns 0..7 (36 products) each led by one extra product 38*h_k
     (2^256 == 38 mod p), so no separate reduction pass is needed; the small
     leading product also cannot overflow the carried-in accumulator;
  3. the overflow V above bit 256 (< 2^37) and bit 255 are folded once with
     2^255 == 19: result < 2^255 + 2^43.
Each column accumulates in a 64-bit VGPR pair with v_mad_u64_u32 and counts
carry-outs (vcc) into the high word of the *next* column's pair, so the
column shift costs two v_mov.  64-bit VGPR tuples must be even-aligned on
gfx950 and inline asm cannot name the halves of a compiler-allocated pair,
so the two accumulator pairs are fixed scratch VGPRs (declared clobbered).
"""
import os
import sys

SCRATCH_BASE = int(os.environ.get("FE_SCRATCH_BASE", "252"))   # v[B:B+3], B even


class Pair:
    def __init__(self, base):
        self.base = base

    @property
    def reg(self):
        return f"v[{self.base}:{self.base + 1}]"

    @property
    def lo(self):
        return f"v{self.base}"

    @property
    def hi(self):
        return f"v{self.base + 1}"


def gen_mul(base=SCRATCH_BASE):
    """Return (asm_lines, operand layout).  Operands:
    %0..%7 r (out), %8..%15 h (scratch out), %16..%23 a (in), %24..%31 b (in)."""
    R = [f"%{i}" for i in range(8)]
    H = [f"%{8 + i}" for i in range(8)]
    A = [f"%{16 + i}" for i in range(8)]
    B = [f"%{24 + i}" for i in range(8)]
    P, Q = Pair(base), Pair(base + 2)
    L = []
    cur, nxt = P, Q
    first = True

    def column(prods, out_reg, first_is_small):
        """Accumulate one column.  The carried-in accumulator is < 10*2^32, so a
        full 32x32 first product CAN overflow 2^64 (all-ones limbs); only a first
        product that is small (38*h < 2^38) or a chain start (src2 = 0) cannot."""
        nonlocal cur, nxt, first
        counted = False
        for idx, (x, y) in enumerate(prods):
            safe = first or (idx == 0 and first_is_small)
            src2 = "0" if first else cur.reg
            first = False
            L.append(f"v_mad_u64_u32 {cur.reg}, vcc, {x}, {y}, {src2}")
            if safe:
                continue
            if not counted:
                L.append(f"v_addc_co_u32 {nxt.hi}, vcc, 0, 0, vcc")
                counted = True
            else:
                L.append(f"v_addc_co_u32 {nxt.hi}, vcc, 0, {nxt.hi}, vcc")
        if not counted:
            L.append(f"v_mov_b32 {nxt.hi}, 0")
        L.append(f"v_mov_b32 {out_reg}, {cur.lo}")
        L.append(f"v_mov_b32 {nxt.lo}, {cur.hi}")
        cur, nxt = nxt, cur

    # 1. high columns 8..14 -> h0..h6, h7 = final carry word
    for k in range(8, 15):
        column([(A[i], B[k - i]) for i in range(k - 7, 8)], H[k - 8], False)
    L.append(f"v_mov_b32 {H[7]}, {cur.lo}")
    # 2. low columns 0..7 with 38*h_k folded in
    first = True
    for k in range(8):
        column([(H[k], "38")] + [(A[i], B[k - i]) for i in range(k + 1)], R[k], True)
    # cur = V (overflow above 2^256, < 2^37). 3. fold bits >= 255 with 19.
    V = cur
    T = nxt   # free pair: T.lo = top_lo, T.hi = top_hi, then reused for 19*top
    L.append(f"v_alignbit_b32 {T.lo}, {V.lo}, {R[7]}, 31")
    L.append(f"v_alignbit_b32 {T.hi}, {V.hi}, {V.lo}, 31")
    L.append(f"v_and_b32 {R[7]}, 0x7fffffff, {R[7]}")
    L.append(f"v_mad_u64_u32 {V.reg}, vcc, {T.lo}, 19, 0")       # V = 19*top_lo (64-bit)
    L.append(f"v_mad_u32_u24 {V.hi}, {T.hi}, 19, {V.hi}")         # V += 19*top_hi << 32 (top_hi < 2^6)
    L.append(f"v_add_co_u32 {R[0]}, vcc, {R[0]}, {V.lo}")
    L.append(f"v_addc_co_u32 {R[1]}, vcc, {R[1]}, {V.hi}, vcc")
    for i in range(2, 8):
        L.append(f"v_addc_co_u32 {R[i]}, vcc, 0, {R[i]}, vcc")
    return L


def gen_add():
    """r = a + b (loose inputs) -> tight.  %0..%7 r, %8 t (scratch), %9..%16 a, %17..%24 b."""
    R = [f"%{i}" for i in range(8)]
    t = "%8"
    A = [f"%{9 + i}" for i in range(8)]
    B = [f"%{17 + i}" for i in range(8)]
    L = [f"v_add_co_u32 {R[0]}, vcc, {A[0]}, {B[0]}"]
    for i in range(1, 8):
        L.append(f"v_addc_co_u32 {R[i]}, vcc, {A[i]}, {B[i]}, vcc")
    L.append(f"v_addc_co_u32 {t}, vcc, 0, 0, vcc")            # carry c
    L.append(f"v_alignbit_b32 {t}, {t}, {R[7]}, 31")               # top = 2c + bit255 (<= 3)
    L.append(f"v_and_b32 {R[7]}, 0x7fffffff, {R[7]}")
    L.append(f"v_mul_u32_u24 {t}, 19, {t}")
    L.append(f"v_add_co_u32 {R[0]}, vcc, {R[0]}, {t}")
    for i in range(1, 8):
        L.append(f"v_addc_co_u32 {R[i]}, vcc, 0, {R[i]}, vcc")
    return L


def gen_sub():
    """r = a - b (a loose, b tight) -> loose:  a - b, and if it borrowed add 2p = 2^256-38
    (i.e. subtract 38 modulo 2^256; the true value a-b+2p is >= 0 because b is tight).
    %0..%7 r, %8 t (scratch), %9..%16 a, %17..%24 b."""
    R = [f"%{i}" for i in range(8)]
    t = "%8"
    A = [f"%{9 + i}" for i in range(8)]
    B = [f"%{17 + i}" for i in range(8)]
    L = [f"v_sub_co_u32 {R[0]}, vcc, {A[0]}, {B[0]}"]
    for i in range(1, 8):
        L.append(f"v_subb_co_u32 {R[i]}, vcc, {A[i]}, {B[i]}, vcc")
    L.append(f"v_subb_co_u32 {t}, vcc, 0, 0, vcc")             # t = -borrow
    L.append(f"v_and_b32 {t}, 38, {t}")
    L.append(f"v_sub_co_u32 {R[0]}, vcc, {R[0]}, {t}")
    for i in range(1, 8):
        L.append(f"v_subbrev_co_u32 {R[i]}, vcc, 0, {R[i]}, vcc")
    return L


def emit_fn(name, lines, outs, ins, clobbers, doc):
    body = "\\n\\t".join(lines)
    s = f"/* {doc} */\n"
    s += f"__device__ __forceinline__ void {name}( {', '.join(outs[0] + ins[0])} ) {{\n"
    s += f'  asm( "{body}"\n'
    s += f"       : {', '.join(outs[1])}\n"
    s += f"       : {', '.join(ins[1])}\n"
    s += f"       : {', '.join(clobbers)} );\n}}\n\n"
    return s


def main(out_path):
    base = SCRATCH_BASE
    clob_mul = [f'"v{base + i}"' for i in range(4)] + ['"vcc"']
    hdr = [
        "/* fe25519_asm.h -- GENERATED by gen_fe_asm.py; do not edit.",
        "   GF(2^255-19) on 8x32-bit limbs for gfx950 (see gen_fe_asm.py for the schedule).",
        f"   Fixed scratch VGPRs: v{base}..v{base + 3} (clobbered by fe_mul). */",
        "#pragma once",
        "#include <stdint.h>",
        "",
        f"#define FE_ASM_SCRATCH_BASE {base}",
        "",
    ]
    s = "\n".join(hdr) + "\n"
    # fe_mul
    outs = (["uint32_t r[8]"], [f'"=&v"(r[{i}])' for i in range(8)])
    mul_ins_decl = ["uint32_t const a[8]", "uint32_t const b[8]"]
    mul_ops = ([f'"=&v"(h[{i}])' for i in range(8)] + [f'"v"(a[{i}])' for i in range(8)] +
               [f'"v"(b[{i}])' for i in range(8)])
    body = "\\n\\t".join(gen_mul(base))
    s += "/* r = a*b mod p: loose x loose -> tight (< 2^255 + 2^43). */\n"
    s += "__device__ __forceinline__ void fe_mul( uint32_t r[8], uint32_t const a[8], uint32_t const b[8] ) {\n"
    s += "  uint32_t h[8];\n"
    s += f'  asm( "{body}"\n'
    s += f"       : {', '.join(outs[1] + mul_ops[:8])}\n"
    s += f"       : {', '.join(mul_ops[8:])}\n"
    s += f"       : {', '.join(clob_mul)} );\n}}\n\n"
    rq = ['"=&v"(r[%d])' % i for i in range(8)] + ['"=&v"(t)']
    aq = ['"v"(a[%d])' % i for i in range(8)] + ['"v"(b[%d])' % i for i in range(8)]
    for name, gen, doc in (("fe_add", gen_add, "r = a + b: loose + loose -> tight."),
                           ("fe_sub", gen_sub, "r = a - b: loose - tight -> loose.")):
        body = "\\n\\t".join(gen())
        s += "/* %s */\n" % doc
        s += "__device__ __forceinline__ void %s( uint32_t r[8], uint32_t const a[8], uint32_t const b[8] ) {\n" % name
        s += "  uint32_t t;\n"
        s += '  asm( "%s"\n' % body
        s += "       : %s\n" % ", ".join(rq)
        s += "       : %s\n" % ", ".join(aq)
        s += '       : "vcc" );\n}\n\n'
    with open(out_path, "w") as f:
        f.write(s)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(os.path.abspath(__file__)), "fe25519_asm.h"))
