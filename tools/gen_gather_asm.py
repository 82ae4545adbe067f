#!/usr/bin/env python3
"""Generate csrc/gather_asm.inc -- the inner loop of kernel K1 (k_stream).

Why generated: the loop is a fully unrolled, software-pipelined sequence of
16 positions (two 64-entry blocks of 8-entry batches) whose register names
are static per position; writing it by hand is error-prone.

Per batch p (8 stream entries {sign, word1}):
  ISSUE(p): v_readlane word1/sign of the 8 entries from the lane-parallel
            entry block (VGPR pair A = v240/v241 or B = v242/v243) into the
            SGPR set p%2 (s36..s51 / s52..s67); v_bfi the per-lane LDS
            address (word1's row bits + lane*16); 8 ds_read_b128 into the
            X set p%2 (v168..v199 / v200..v231).
  FMA(p):   s_waitcnt lgkmcnt(8) (the 8 reads of batch p+1 stay in flight),
            s_set_gpr_idx_on/idx word1 (low 8 bits = 4*slot) then two
            v_pk_fma_f32 acc[slot] += sign * x (DST and SRC2 relatively
            addressed), s_set_gpr_idx_off.
Position p does ISSUE(p) then FMA(p-1), so a batch's LDS latency hides
under the previous batch's FMAs and other waves.  Entry blocks come from
global memory (vmcnt, in order -- unlike SMEM, which shares lgkmcnt with LDS
and returns out of order); the next block is prefetched at each block start.

Registers: acc v40..v167 (pinned asm operands), X v168..v231 (each LDS
address is computed into the first register of its destination quad),
entry blocks v232..v235, block offset v236; SGPR sets s36..s67; s68 holds
the caller's M0 (s_set_gpr_idx_* overwrites it) and is restored on exit.
"""
import os
import sys

SETS = {0: 36, 1: 52}          # SGPR set base: pair i = (s[base+2i] sign, s[base+2i+1] word1)
XSET = {0: 168, 1: 200}        # X set base: entry i -> v[base+4i : base+4i+3]
# entry block VGPRs (sign, word1): block A is the chunk's first block, which
# the previous chunk's gather prefetched; it alternates between v232/v233 and
# v238/v239 with the chunk parity (PAR), the other pair receives the next
# chunk's first block.  Block B is internal.
EBLK_A = {0: (232, 233), 1: (238, 239)}  # VGPR tuples must be even-aligned
EBLK = {0: EBLK_A[0], 1: (234, 235)}
VOFF = "v236"
PAR = 0


ABL = 0  # ablation (timing experiments only; results are wrong for ABL != 0)


def issue(p):
    blk = (p // 8) % 2
    s = SETS[p % 2]
    x = XSET[p % 2]
    vsgn, vw1 = EBLK[blk]
    lane0 = 8 * (p % 8)
    out = []
    for i in range(8):
        if ABL == 2:
            out.append(f"s_mov_b32 s{s + 2 * i + 1}, {4 * i}")
        else:
            out.append(f"v_readlane_b32 s{s + 2 * i + 1}, v{vw1}, {lane0 + i}")
    for i in range(8):
        if ABL == 2:
            out.append(f"s_mov_b32 s{s + 2 * i}, 1.0")
        else:
            out.append(f"v_readlane_b32 s{s + 2 * i}, v{vsgn}, {lane0 + i}")
    # the address goes into the first register of the destination quad
    for i in range(8):
        out.append(f"v_bfi_b32 v{x + 4 * i}, %[mask], %[lane], s{s + 2 * i + 1}")
    for i in range(8):
        if ABL != 3:
            out.append(f"ds_read_b128 v[{x + 4 * i}:{x + 4 * i + 3}], v{x + 4 * i}")
    return out


def fma(parity, wait):
    s = SETS[parity]
    x = XSET[parity]
    out = [f"s_waitcnt lgkmcnt({wait})"]
    if ABL == 4:
        return out
    for i in range(8):
        w1 = f"s{s + 2 * i + 1}"
        pair = f"s[{s + 2 * i}:{s + 2 * i + 1}]"
        a = 40 + 4 * i if ABL == 1 else 40
        if ABL != 1:
            out.append(f"s_set_gpr_idx_on {w1}, gpr_idx(SRC2,DST)" if i == 0 else f"s_set_gpr_idx_idx {w1}")
        out.append(f"v_pk_fma_f32 v[{a}:{a + 1}], v[{x + 4 * i}:{x + 4 * i + 1}], {pair}, v[{a}:{a + 1}] op_sel_hi:[1,0,1]")
        out.append(f"v_pk_fma_f32 v[{a + 2}:{a + 3}], v[{x + 4 * i + 2}:{x + 4 * i + 3}], {pair}, v[{a + 2}:{a + 3}] op_sel_hi:[1,0,1]")
    if ABL != 1:
        out.append("s_set_gpr_idx_off")
    return out


def prefetch(into_blk):
    """At a block start with more than 8 batches left: load the next block."""
    vsgn, vw1 = EBLK[into_blk]
    assert vw1 == vsgn + 1
    return [
        "s_cmp_gt_u32 %[nb], 8",
        "s_cbranch_scc0 .Lnopf{P}%=",
        f"v_add_u32 {VOFF}, 0x200, {VOFF}",
        f"global_load_dwordx2 v[{vsgn}:{vw1}], {VOFF}, %[ent]",
        ".Lnopf{P}%=:",
    ]


def step_end(p):
    """Count the batch; on the last one drain the pipeline."""
    return [
        "s_sub_u32 %[nb], %[nb], 1",
        "s_cmp_eq_u32 %[nb], 0",
        f"s_cbranch_scc1 .Ldrain{p % 2}%=",
    ]


def generate():
    na = EBLK_A[1 - PAR]
    L = ["s_mov_b32 s68, m0"]  # M0 also addresses the caller's LDS-DMA
    # next chunk's first entry block (VOFF = lane*8 on entry)
    L.append(f"global_load_dwordx2 v[{na[0]}:{na[1]}], {VOFF}, %[nent]")
    L.append("s_cmp_eq_u32 %[nb], 0")
    L.append("s_cbranch_scc1 .Lend%=")
    # prologue: block A is the caller-provided input; maybe prefetch block B
    L += [l.replace("{P}", "pro") for l in prefetch(1)]
    L += issue(0)
    L += step_end(0)
    L.append("s_branch .Lp1%=")
    L.append(".Ltop%=:")
    for p in range(16):
        if p == 1:
            L.append(".Lp1%=:")
        if p % 8 == 0:
            L.append("s_waitcnt vmcnt(0)")  # this block's entries have landed
            L += [l.replace("{P}", str(p)) for l in prefetch(1 - (p // 8))]
        L += issue(p)
        L += fma((p - 1) % 2, 8)
        L += step_end(p)
    L.append("s_branch .Ltop%=")
    for par in (0, 1):
        L.append(f".Ldrain{par}%=:")
        L += fma(par, 0)
        if par == 0:
            L.append("s_branch .Lend%=")
    L.append(".Lend%=:")
    L.append("s_mov_b32 m0, s68")
    return L


def emit(f, lines):
    f.write(f"#define TCSC_GATHER_ASM_{PAR} \\\n")
    for l in lines:
        f.write(f'    "{l}\\n\\t" \\\n')
    f.write('    ""\n')


def main():
    global ABL, PAR, EBLK
    here = os.path.dirname(os.path.abspath(__file__))
    out = os.path.join(here, "..", "sparse-matrix-multiplication-benchmark_amd", "csrc", "gather_asm.inc")
    with open(out, "w") as f:
        f.write("// GENERATED by tools/gen_gather_asm.py -- do not edit by hand.\n")
        f.write("// See the generator's docstring for the schedule.  TCSC_ABLATION != 0\n")
        f.write("// selects timing-only variants (wrong results) for experiments.\n")
        f.write("#if !defined(TCSC_ABLATION) || TCSC_ABLATION == 0 || TCSC_ABLATION >= 6\n")
        for a in (0, 1, 2, 3, 4, 5):
            if a:
                f.write(f"#elif TCSC_ABLATION == {a}\n")
            ABL = a
            for PAR in (0, 1):
                EBLK = {0: EBLK_A[PAR], 1: (234, 235)}
                if a == 5:  # no gather at all: only the M0 save and next-block load
                    emit(f, generate()[:2] + ["s_mov_b32 m0, s68"])
                else:
                    emit(f, generate())
        f.write("#endif\n")
    print(out)


if __name__ == "__main__":
    sys.exit(main())
