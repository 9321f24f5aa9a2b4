"""Generate tools/fe_cs.h: a carry-save column variant of coa_fe.h's field
product as a few large inline-asm statements (measured and rejected: it
issues fewer instructions but more mads, and runs 9 % slower per multiply at
one wave per SIMD, profiles/r02_ubench_fecs.txt).

Each 32x32 partial product of a column goes into that column's own fresh
64-bit accumulator (v_mad_u64_u32, the column's first product adds 0 and
cannot carry) and the mad carry-outs into the column's carry word, so no
accumulator has to be shifted into a new register pair between columns (the
odd half of a pair cannot start an even-aligned pair: the old comba paid a
v_mov per column for that, plus one per zero-extension of the reduction).
The columns 8..14 are then folded into 0..7 as 64-bit mads by 38, and two
carry chains produce the words.  All columns of a product are one asm
statement, because hipcc places an `s_nop 0` in front of every inline-asm
statement that follows another.

usage: python tools/gen_fe_cs.py  (rewrites the header in place)
"""
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tools", "fe_cs.h")


def asm_block(lines):
    return "\n".join(f'      "{l}\\n\\t"' for l in lines[:-1]) + f'\n      "{lines[-1]}"'


def mul_columns():
    """One asm: outputs %0..%14 = P0..P14 (u64), %15..%27 = C1..C13;
    inputs %28..%35 = a0..a7, %36..%43 = b0..b7."""
    P = lambda k: f"%{k}"
    C = lambda k: f"%{14 + k}"  # C1 -> %15
    A = lambda i: f"%{28 + i}"
    B = lambda j: f"%{36 + j}"
    lines = []
    for k in range(15):
        pairs = [(i, k - i) for i in range(8) if 0 <= k - i < 8]
        for n, (i, j) in enumerate(pairs):
            if n == 0:
                lines.append(f"v_mad_u64_u32 {P(k)}, vcc, {A(i)}, {B(j)}, 0")
            else:
                lines.append(f"v_mad_u64_u32 {P(k)}, vcc, {A(i)}, {B(j)}, {P(k)}")
                if n == 1:
                    lines.append(f"v_cndmask_b32_e64 {C(k)}, 0, 1, vcc")
                else:
                    lines.append(f"v_addc_co_u32_e32 {C(k)}, vcc, 0, {C(k)}, vcc")
    outs = ", ".join([f'"=&v"(P[{k}])' for k in range(15)] + [f'"=&v"(C[{k}])' for k in range(1, 14)])
    ins = ", ".join([f'"v"(a.v[{i}])' for i in range(8)] + [f'"v"(b.v[{j}])' for j in range(8)])
    return lines, outs, ins


def sq_columns():
    """Cross products i < j.  One asm: outputs %0..%12 = P1..P13, %13..%21 =
    C3..C11; inputs %22..%29 = a0..a7."""
    P = lambda k: f"%{k - 1}"
    C = lambda k: f"%{13 + k - 3}"
    A = lambda i: f"%{22 + i}"
    lines = []
    for k in range(1, 14):
        pairs = [(i, k - i) for i in range(8) if 0 <= k - i < 8 and i < k - i]
        for n, (i, j) in enumerate(pairs):
            if n == 0:
                lines.append(f"v_mad_u64_u32 {P(k)}, vcc, {A(i)}, {A(j)}, 0")
            else:
                lines.append(f"v_mad_u64_u32 {P(k)}, vcc, {A(i)}, {A(j)}, {P(k)}")
                lines.append(f"v_cndmask_b32_e64 {C(k)}, 0, 1, vcc" if n == 1 else
                             f"v_addc_co_u32_e32 {C(k)}, vcc, 0, {C(k)}, vcc")
    outs = ", ".join([f'"=&v"(X[{k}])' for k in range(1, 14)] + [f'"=&v"(XC[{k}])' for k in range(3, 12)])
    ins = ", ".join(f'"v"(a.v[{i}])' for i in range(8))
    return lines, outs, ins


def sq_double():
    """2 * cross + diagonal.  Outputs %0..%14 = P0..P14, %15..%27 = C1..C13;
    inputs %28..%40 = X1..X13 (u64), %41..%53 = hi(X1..X13), %54..%62 =
    XC3..XC11, %63..%70 = a0..a7."""
    P = lambda k: f"%{k}"
    C = lambda k: f"%{14 + k}"
    X = lambda k: f"%{28 + k - 1}"
    XH = lambda k: f"%{41 + k - 1}"
    XC = lambda k: f"%{54 + k - 3}"
    A = lambda i: f"%{63 + i}"
    lines = []
    for k in range(15):
        if 1 <= k <= 13:
            if 3 <= k <= 11:
                lines.append(f"v_alignbit_b32 {C(k)}, {XC(k)}, {XH(k)}, 31")
            else:
                lines.append(f"v_lshrrev_b32_e32 {C(k)}, 31, {XH(k)}")
            lines.append(f"v_lshlrev_b64 {P(k)}, 1, {X(k)}")
        if k % 2 == 0:
            i = k // 2
            if k in (0, 14):
                lines.append(f"v_mad_u64_u32 {P(k)}, vcc, {A(i)}, {A(i)}, 0")
            else:
                lines.append(f"v_mad_u64_u32 {P(k)}, vcc, {A(i)}, {A(i)}, {P(k)}")
                lines.append(f"v_addc_co_u32_e32 {C(k)}, vcc, 0, {C(k)}, vcc")
    outs = ", ".join([f'"=&v"(P[{k}])' for k in range(15)] + [f'"=&v"(C[{k}])' for k in range(1, 14)])
    ins = ", ".join([f'"v"(X[{k}])' for k in range(1, 14)] + [f'"v"((uint32_t)(X[{k}] >> 32))' for k in range(1, 14)]
                    + [f'"v"(XC[{k}])' for k in range(3, 12)] + [f'"v"(a.v[{i}])' for i in range(8)])
    return lines, outs, ins


def fold():
    """Columns 8..14 into 0..7.  Outputs %0..%7 P0..P7 (+), %8 C0 (=),
    %9..%15 C1..C7 (+); inputs %16..%22 lo(P8..P14), %23..%29 hi(P8..P14),
    %30..%35 C8..C13."""
    P = lambda k: f"%{k}"
    C = lambda k: f"%{8 + k}"
    LO = lambda k: f"%{16 + k - 8}"
    HI = lambda k: f"%{23 + k - 8}"
    CH = lambda k: f"%{30 + k - 8}"
    lines = []
    for k in range(8, 15):
        lo, hi = k - 8, k - 7
        lines.append(f"v_mad_u64_u32 {P(lo)}, vcc, {LO(k)}, 38, {P(lo)}")
        lines.append(f"v_cndmask_b32_e64 {C(lo)}, 0, 1, vcc" if lo == 0 else
                     f"v_addc_co_u32_e32 {C(lo)}, vcc, 0, {C(lo)}, vcc")
        lines.append(f"v_mad_u64_u32 {P(hi)}, vcc, {HI(k)}, 38, {P(hi)}")
        lines.append(f"v_addc_co_u32_e32 {C(hi)}, vcc, 0, {C(hi)}, vcc")
        if k <= 13:
            lines.append(f"v_mad_u32_u24 {C(lo)}, {CH(k)}, 38, {C(lo)}")
    outs = ", ".join([f'"+v"(P[{k}])' for k in range(8)] + ['"=&v"(C[0])'] + [f'"+v"(C[{k}])' for k in range(1, 8)])
    ins = ", ".join([f'"v"((uint32_t)P[{k}])' for k in range(8, 15)] + [f'"v"((uint32_t)(P[{k}] >> 32))' for k in range(8, 15)]
                    + [f'"v"(C[{k}])' for k in range(8, 14)])
    return lines, outs, ins


def tail():
    """Outputs %0..%7 r, %8 w8, %9 w9, %10 t1, %11 t2; inputs %12..%19
    lo(P0..P7), %20..%27 hi(P0..P7), %28..%35 C0..C7."""
    R = lambda k: f"%{k}"
    LO = lambda k: f"%{12 + k}"
    HI = lambda k: f"%{20 + k}"
    C = lambda k: f"%{28 + k}"
    L = [f"v_add_co_u32_e32 {R(1)}, vcc, {LO(1)}, {HI(0)}"]
    for k in range(2, 8):
        L.append(f"v_addc_co_u32_e32 {R(k)}, vcc, {LO(k)}, {HI(k - 1)}, vcc")
    L.append(f"v_addc_co_u32_e32 %8, vcc, 0, {HI(7)}, vcc")
    L.append(f"v_addc_co_u32_e32 %9, vcc, 0, {C(7)}, vcc")
    L.append(f"v_add_co_u32_e32 {R(2)}, vcc, {R(2)}, {C(0)}")
    for k in range(3, 8):
        L.append(f"v_addc_co_u32_e32 {R(k)}, vcc, {R(k)}, {C(k - 2)}, vcc")
    L.append(f"v_addc_co_u32_e32 %8, vcc, %8, {C(6)}, vcc")
    L.append("v_addc_co_u32_e32 %9, vcc, 0, %9, vcc")
    # 38 * (w8 + 2^32 w9) into words 0..1
    L += ["v_mul_lo_u32 %10, %8, 38", "v_mul_hi_u32 %11, %8, 38", "v_mad_u32_u24 %11, %9, 38, %11",
          f"v_add_co_u32_e32 {R(0)}, vcc, {LO(0)}, %10", f"v_addc_co_u32_e32 {R(1)}, vcc, {R(1)}, %11, vcc",
          "s_cbranch_vccz 1f"]
    for k in range(2, 8):
        L.append(f"v_addc_co_u32_e32 {R(k)}, vcc, 0, {R(k)}, vcc")
    L += ["v_cndmask_b32_e64 %10, 0, 38, vcc", f"v_add_u32_e32 {R(0)}, {R(0)}, %10"]
    outs = ", ".join([f'"=&v"(r.v[{k}])' for k in range(8)] + ['"=&v"(w8)', '"=&v"(w9)', '"=&v"(t1)', '"=&v"(t2)'])
    ins = ", ".join([f'"v"((uint32_t)P[{k}])' for k in range(8)] + [f'"v"((uint32_t)(P[{k}] >> 32))' for k in range(8)]
                    + [f'"v"(C[{k}])' for k in range(8)])
    return L, outs, ins


def stmt(lines, outs, ins, label=False):
    body = asm_block(lines)
    if label:
        body = body + '\n      "\\n1:"'
    return f"  asm({body[6:]}\n      : {outs}\n      : {ins}\n      : \"vcc\");\n"


def main():
    mc = mul_columns()
    sc = sq_columns()
    sd = sq_double()
    fo = fold()
    ta = tail()
    hdr = f'''// GENERATED by tools/gen_fe_cs.py -- do not edit by hand.
//
// Carry-save column products (fecs::mul / fecs::sq), an A/B variant of
// coa_fe.h's comba for tools/ubench_fecs.hip; see the generator's docstring.  Value bookkeeping: column k is
// P[k] + 2^64 C[k] (C[k] <= 7); folding 8..14 by 38 leaves C[k] <= 237 for
// k < 8; the tail's top word pair T = w8 + 2^32 w9 is < 2^42, so 38 T < 2^48
// is one 64-bit add into words 0..1.  Its carry past word 1 (probability
// ~2^-17 per lane) runs the propagation behind a wave-uniform
// s_cbranch_vccz; a carry out of word 7 then adds 38 to word 0, which cannot
// carry again (the words are all zero after such a wrap).
#pragma once
#include "../xrpl-coa-prototype_amd/csrc/coa_fe.h"

namespace fecs {{

COA_DEV void fold_high(uint64_t* P, uint32_t* C) {{
{stmt(*fo)}}}

COA_DEV void tail(fe& r, const uint64_t* P, const uint32_t* C) {{
  uint32_t w8, w9, t1, t2;
{stmt(*ta, label=True)}}}

COA_DEV void mul(fe& r, const fe& a, const fe& b) {{
  uint64_t P[15];
  uint32_t C[15];
{stmt(*mc)}  fold_high(P, C);
  tail(r, P, C);
}}

COA_DEV void sq(fe& r, const fe& a) {{
  uint64_t X[14], P[15];
  uint32_t XC[12], C[15];
{stmt(*sc)}{stmt(*sd)}  fold_high(P, C);
  tail(r, P, C);
}}

}}  // namespace fecs
'''
    with open(OUT, "w") as f:
        f.write(hdr)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
