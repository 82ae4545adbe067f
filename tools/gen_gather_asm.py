#!/usr/bin/env python3
"""Generate the gather loop of kernel K1 (k_stream) for one register geometry.

    gen_gather_asm.py [--cw 16] [--batch 4] [--nset 2] [--budget 128] [-o path]

Why generated: the loop is a fully unrolled, software-pipelined sequence of
positions (two 64-entry blocks of BATCH-entry batches) whose register names
are static per position; writing it by hand is error-prone, and the kernel's
geometry is a tuning knob: columns per wave CW (4*CW accumulator VGPRs),
batch size, pipeline depth NSET and the VGPR budget per wave (512 / waves
per SIMD).

Per batch p (BATCH stream entries {sign, word1}):
  ISSUE(p): v_readlane word1/sign of the batch's entries from the
            lane-parallel entry block (VGPR pair A or B) into SGPR set
            p % NSET; v_bfi the per-lane LDS address (word1's row bits +
            lane*16) into the first register of the entry's X quad;
            ds_read_b128 into that quad.
  FMA(p):   s_waitcnt lgkmcnt(BATCH*(NSET-1)) (a later batch's reads stay in
            flight), s_set_gpr_idx_on/idx word1 (low 8 bits = 4*slot), two
            v_pk_fma_f32 acc[slot] += sign * x (DST and SRC2 relatively
            addressed), s_set_gpr_idx_off.
NSET = 2: position p does ISSUE(p) then FMA(p-1), so a batch's LDS latency
hides under the previous batch's FMAs.  NSET = 1: ISSUE(p) then FMA(p); the
latency is hidden by the SIMD's other waves instead (more of them fit).
Entry blocks come from global memory (vmcnt, in order); the next block is
prefetched at each block start.  The chunk's first block (pair A, which
alternates between two pinned pairs with the chunk parity PAR) was loaded by
the previous chunk's gather; this gather begins by loading the NEXT chunk's
first block into the other pair.

s68 keeps the caller's M0 (s_set_gpr_idx_* overwrites it and the caller's
LDS-DMA uses it) and is restored on exit.  SGPR sets start at s36.

The output defines TCSC_GATHER_ASM_0/1 (chunk parity), the pinned operand
lists (TCSC_ACC_OPERANDS, TCSC_E0S/E0W/E1S/E1W/VOFF), TCSC_GATHER_CLOBBERS
and TCSC_GEN_* (the kernel static_asserts its geometry against them).
TCSC_ABLATION = 1..5 selects timing-only variants (wrong results):
1 no index mode, 2 no readlane, 3 no LDS read, 4 no FMA, 5 no gather.
"""
import argparse
import os
import sys


class Geo:
    def __init__(self, cw, batch, nset, budget):
        assert cw % 8 == 0 and 64 % batch == 0 and nset in (1, 2)
        self.cw, self.batch, self.nset, self.budget = cw, batch, nset, budget
        self.ppb = 64 // batch  # positions per 64-entry block
        nacc, nx = 4 * cw, 4 * batch * nset
        # pinned block at the top of the budget: acc | X sets | A0 A1 B | voff
        self.voff = budget - 1
        e = (budget - 1) & ~1
        self.eb = (e - 2, e - 1)
        self.ea = {0: (e - 6, e - 5), 1: (e - 4, e - 3)}
        self.xbase = ((e - 6) - nx) & ~3
        self.acc = (self.xbase - nacc) & ~1
        assert self.acc >= 20, "VGPR budget too small for this geometry"
        self.xset = {s: self.xbase + 4 * batch * s for s in range(nset)}
        self.sset = {s: 36 + 2 * batch * s for s in range(nset)}
        self.slast = 36 + 2 * batch * nset - 1
        assert self.slast < 68


ABL = 0


def issue(g, p, eblk):
    vsgn, vw1 = eblk[(p // g.ppb) % 2]
    s, x = g.sset[p % g.nset], g.xset[p % g.nset]
    lane0 = g.batch * (p % g.ppb)
    out = []
    for i in range(g.batch):
        out.append(f"s_mov_b32 s{s + 2 * i + 1}, {4 * (i % g.cw)}" if ABL == 2 else
                   f"v_readlane_b32 s{s + 2 * i + 1}, v{vw1}, {lane0 + i}")
    for i in range(g.batch):
        out.append(f"s_mov_b32 s{s + 2 * i}, 1.0" if ABL == 2 else
                   f"v_readlane_b32 s{s + 2 * i}, v{vsgn}, {lane0 + i}")
    for i in range(g.batch):
        out.append(f"v_bfi_b32 v{x + 4 * i}, %[mask], %[lane], s{s + 2 * i + 1}")
    if ABL != 3:
        for i in range(g.batch):
            out.append(f"ds_read_b128 v[{x + 4 * i}:{x + 4 * i + 3}], v{x + 4 * i}")
    return out


def fma(g, sidx, wait):
    s, x = g.sset[sidx], g.xset[sidx]
    out = [f"s_waitcnt lgkmcnt({wait})"]
    if ABL == 4:
        return out
    for i in range(g.batch):
        w1, pair = f"s{s + 2 * i + 1}", f"s[{s + 2 * i}:{s + 2 * i + 1}]"
        a = g.acc + 4 * (i % g.cw) if ABL == 1 else g.acc
        if ABL != 1:
            out.append(f"s_set_gpr_idx_on {w1}, gpr_idx(SRC2,DST)" if i == 0 else f"s_set_gpr_idx_idx {w1}")
        out.append(f"v_pk_fma_f32 v[{a}:{a + 1}], v[{x + 4 * i}:{x + 4 * i + 1}], {pair}, v[{a}:{a + 1}] op_sel_hi:[1,0,1]")
        out.append(f"v_pk_fma_f32 v[{a + 2}:{a + 3}], v[{x + 4 * i + 2}:{x + 4 * i + 3}], {pair}, v[{a + 2}:{a + 3}] op_sel_hi:[1,0,1]")
    if ABL != 1:
        out.append("s_set_gpr_idx_off")
    return out


def prefetch(g, eblk, into_blk, tag):
    """At a block start with batches left beyond this block: load the next block."""
    vsgn, vw1 = eblk[into_blk]
    return [
        f"s_cmp_gt_u32 %[nb], {g.ppb}",
        f"s_cbranch_scc0 .Lnopf{tag}%=",
        f"v_add_u32 v{g.voff}, 0x200, v{g.voff}",
        f"global_load_dwordx2 v[{vsgn}:{vw1}], v{g.voff}, %[ent]",
        f".Lnopf{tag}%=:",
    ]


def count(target):
    return ["s_sub_u32 %[nb], %[nb], 1", "s_cmp_eq_u32 %[nb], 0", f"s_cbranch_scc1 {target}"]


def generate(g, par):
    eblk = {0: g.ea[par], 1: g.eb}
    na = g.ea[1 - par]
    L = ["s_mov_b32 s68, m0",
         f"global_load_dwordx2 v[{na[0]}:{na[1]}], v{g.voff}, %[nent]"]  # next chunk's first block
    if ABL == 5:
        return L + ["s_mov_b32 m0, s68"]
    L += ["s_cmp_eq_u32 %[nb], 0", "s_cbranch_scc1 .Lend%="]
    L += prefetch(g, eblk, 1, "pro")
    npos = 2 * g.ppb
    if g.nset == 2:
        L += issue(g, 0, eblk)
        L += count(".Ldrain0%=")
        L.append("s_branch .Lp1%=")
        L.append(".Ltop%=:")
        for p in range(npos):
            if p == 1:
                L.append(".Lp1%=:")
            if p % g.ppb == 0:
                L.append("s_waitcnt vmcnt(0)")  # this block's entries have landed
                L += prefetch(g, eblk, 1 - p // g.ppb, str(p))
            L += issue(g, p, eblk)
            L += fma(g, (p - 1) % 2, g.batch)
            L += count(f".Ldrain{p % 2}%=")
        L.append("s_branch .Ltop%=")
        L.append(".Ldrain0%=:")
        L += fma(g, 0, 0)
        L.append("s_branch .Lend%=")
        L.append(".Ldrain1%=:")
        L += fma(g, 1, 0)
    else:
        L.append("s_branch .Lp0%=")
        L.append(".Ltop%=:")
        for p in range(npos):
            if p % g.ppb == 0:
                L.append("s_waitcnt vmcnt(0)")
                L += prefetch(g, eblk, 1 - p // g.ppb, str(p))
            if p == 0:
                L.append(".Lp0%=:")
            L += issue(g, p, eblk)
            L += fma(g, 0, 0)
            L += count(".Lend%=")
        L.append("s_branch .Ltop%=")
    L.append(".Lend%=:")
    L.append("s_mov_b32 m0, s68")
    return L


def emit(f, name, lines):
    f.write(f"#define {name} \\\n")
    for l in lines:
        f.write(f'    "{l}\\n\\t" \\\n')
    f.write('    ""\n')


def write_inc(path, g):
    global ABL
    nvec = 4 * g.cw // 32
    with open(path, "w") as f:
        f.write("// GENERATED by tools/gen_gather_asm.py -- do not edit by hand.\n")
        f.write(f"// geometry: cw={g.cw} batch={g.batch} nset={g.nset} vgpr budget={g.budget}: "
                f"acc v[{g.acc}:{g.acc + 4 * g.cw - 1}], X v[{g.xbase}:{g.xbase + 4 * g.batch * g.nset - 1}], "
                f"A0 v{g.ea[0][0]}:{g.ea[0][1]}, A1 v{g.ea[1][0]}:{g.ea[1][1]}, B v{g.eb[0]}:{g.eb[1]}, "
                f"voff v{g.voff}\n")
        f.write(f"#define TCSC_GEN_CW {g.cw}\n#define TCSC_GEN_BATCH {g.batch}\n#define TCSC_GEN_NSET {g.nset}\n")
        f.write(f"#define TCSC_GEN_BUDGET {g.budget}\n#define TCSC_ACC_VECS {nvec}\n")
        ops = ", ".join(f'"+{{v[{g.acc + 32 * i}:{g.acc + 32 * i + 31}]}}"(acc[{i}])' for i in range(nvec))
        f.write(f"#define TCSC_ACC_OPERANDS(acc) {ops}\n")
        f.write(f'#define TCSC_E0S "+{{v{g.ea[0][0]}}}"\n#define TCSC_E0W "+{{v{g.ea[0][1]}}}"\n')
        f.write(f'#define TCSC_E1S "+{{v{g.ea[1][0]}}}"\n#define TCSC_E1W "+{{v{g.ea[1][1]}}}"\n')
        f.write(f'#define TCSC_E0S_OUT "={{v{g.ea[0][0]}}}"\n#define TCSC_E0W_OUT "={{v{g.ea[0][1]}}}"\n')
        f.write(f'#define TCSC_E0_PAIR "v[{g.ea[0][0]}:{g.ea[0][1]}]"\n')
        f.write(f'#define TCSC_VOFF "+{{v{g.voff}}}"\n')
        clob = ['"memory"', '"scc"']
        clob += [f'"v{r}"' for r in range(g.xbase, g.xbase + 4 * g.batch * g.nset)]
        clob += [f'"v{g.eb[0]}"', f'"v{g.eb[1]}"']
        clob += [f'"s{r}"' for r in range(36, g.slast + 1)] + ['"s68"']
        f.write("#define TCSC_GATHER_CLOBBERS " + ", ".join(clob) + "\n")
        f.write("#if !defined(TCSC_ABLATION) || TCSC_ABLATION == 0 || TCSC_ABLATION >= 6\n")
        for a in (0, 1, 2, 3, 4, 5):
            if a:
                f.write(f"#elif TCSC_ABLATION == {a}\n")
            ABL = a
            for par in (0, 1):
                emit(f, f"TCSC_GATHER_ASM_{par}", generate(g, par))
        f.write("#endif\n")
        ABL = 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cw", type=int, default=16)
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--nset", type=int, default=2)
    ap.add_argument("--budget", type=int, default=128)
    here = os.path.dirname(os.path.abspath(__file__))
    ap.add_argument("-o", default=os.path.join(here, "..", "sparse-matrix-multiplication-benchmark_amd", "csrc",
                                               "gather_asm.inc"))
    a = ap.parse_args()
    write_inc(a.o, Geo(a.cw, a.batch, a.nset, a.budget))
    print(a.o)


if __name__ == "__main__":
    sys.exit(main())
