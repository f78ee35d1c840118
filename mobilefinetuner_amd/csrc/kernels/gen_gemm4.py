#!/usr/bin/env python3
"""Generator of gemm4's hand-scheduled K-tile body (kernels/gemm4_sched.h).

gemm4 (kernels/gemm4.hip) is a 256 x 256 x 64 bf16 GEMM with FOUR waves, one per SIMD, each owning a
128 x 128 accumulator tile (64 blocks of 16 x 16, v_mfma_f32_16x16x32_bf16) held in AGPRs.  One K-tile
(64 deep) is 128 MFMAs per wave in two k-steps of 32; the A/B fragments of a k-step (8 + 8 x 16 B per
lane) are double-buffered in VGPRs (sets 0 / 1), the K-tiles in LDS (two 64 KB buffers filled by
LDS-DMA, buffer_load_dwordx4 ... lds with range-checked descriptors).

The body of one K-tile is ONE inline-asm statement whose instruction order this script fixes
(CDNA HIP guide §5.7: hipcc schedules an asm statement as one opaque instruction), with the
accumulators as tied "+a" operands (the compiler never moves them) and the fragment sets as "+v" /
"=&v" operands whose loads are waited for INSIDE the statement (no VGPR written by an asm load is
visible to the compiler before it landed).  Per K-tile t (buffer cur = t & 1):

  k-step 0 (MFMAs on set 0, fragments of (t, ks 0) read during the previous K-tile):
      16 ds_read_b128 of (t, ks 1) -> set 1, one per READ_GAP MFMAs from MFMA 0
      lgkmcnt(0) + s_barrier before MFMA BAR_A     -> every wave is done reading buffer cur
      16 LDS-DMA pieces of K-tile t + 2 -> buffer cur, one per MFMA from MFMA BAR_A + 1
  k-step 1 (MFMAs on set 1):
      vmcnt(16) + s_barrier before MFMA 64          -> K-tile t + 1 (issued one K-tile ago) landed
      16 ds_read_b128 of (t + 1, ks 0) -> set 0 from buffer cur ^ 1
      lgkmcnt(0) at the end                         -> set 0 complete when the statement ends

Two barriers per K-tile, no LDS-DMA ever waited for before it is one K-tile old, ds_reads always a
whole k-step ahead of their MFMAs.  Layouts: "nt" (A [M, K], B [N, K], both K-contiguous: ds_read_b128
fragments of source-swizzled 128-B rows).

usage: python gen_gemm4.py  (rewrites gemm4_sched.h next to this file)
"""
import os

READ_GAP = 2      # MFMAs between consecutive fragment reads
BAR_A = 40        # MFMA index the "buffer cur free" barrier precedes


def mfma(s, i, j, zero_c=False):
    c = "0" if zero_c else f"%[c{i}{j}]"
    return f"v_mfma_f32_16x16x32_bf16 %[c{i}{j}], %[b{s}_{j}], %[a{s}_{i}], {c}"


def read_order():
    # the first MFMAs of the consuming k-step need A0 and every B
    return [("a", 0)] + [("b", j) for j in range(8)] + [("a", i) for i in range(1, 8)]


def ds_read(s, kind, idx, base):
    return f"ds_read_b128 %[{kind}{s}_{idx}], %[{base}] offset:{idx * 2048}"


def dma(kind, j):
    # piece j of operand kind (A: rows 32 j + 8 w ..; B likewise), LDS dest = m0
    off = (0 if kind == "a" else 32768) + j * 4096
    srd = "srda" if kind == "a" else "srdb"
    return [f"s_add_u32 m0, %[ldsm], {off}", "s_nop 0",
            f"buffer_load_dwordx4 %[o{kind}{j}], %[{srd}], %[koff] offen lds"]


def ktile_nt(read_gap=READ_GAP, bar_a=BAR_A, dma_at=None, with_dma=True, first=False, vm_extra=0):
    """One K-tile: MFMA n = 0..127 (k-step n // 64).  dma_at[q] = the MFMA index (> bar_a) the q-th of
    the 16 LDS-DMA pieces precedes; the ones before MFMA 64 are left in flight by barrier B's vmcnt.
    first: the first K-tile of an output tile (k-step 0 accumulates onto 0, not onto the registers);
    vm_extra: VMEM operations issued between the previous K-tile's DMAs and this one's (the epilogue
    stores of the previous tile in the persistent kernel) that barrier B may leave in flight."""
    if dma_at is None:
        dma_at = list(range(bar_a + 1, bar_a + 17))
    assert len(dma_at) == 16 and min(dma_at) > bar_a and max(dma_at) < 128
    lines = ["s_nop 4"]
    order = [(i, j) for i in range(8) for j in range(8)]
    reads = read_order()
    dmas = [dma("a", j) for j in range(8)] + [dma("b", j) for j in range(8)]
    at = {n: q for q, n in enumerate(dma_at)}
    before_b = sum(1 for n in dma_at if n < 64)
    for n in range(128):
        ks, (i, j) = n // 64, order[n % 64]
        m = n % 64
        if n == 64:
            lines += [f"s_waitcnt vmcnt({min(63, before_b + vm_extra)})", "s_barrier",
                      "v_xor_b32 %[ra0], 0x10000, %[ra0]", "v_xor_b32 %[rb0], 0x10000, %[rb0]"]
        if m % read_gap == 0 and m // read_gap < len(reads):
            kind, idx = reads[m // read_gap]
            if ks == 0:
                lines.append(ds_read(1, kind, idx, "ra1" if kind == "a" else "rb1"))
            else:
                lines.append(ds_read(0, kind, idx, "ra0" if kind == "a" else "rb0"))
        if n == bar_a:
            lines += ["s_waitcnt lgkmcnt(0)", "s_barrier"]
        if n in at and with_dma:
            lines += dmas[at[n]]
        lines.append(mfma(ks, i, j, zero_c=first and ks == 0))
    lines += ["v_xor_b32 %[ra1], 0x10000, %[ra1]", "v_xor_b32 %[rb1], 0x10000, %[rb1]", "s_waitcnt lgkmcnt(0)"]
    return lines


def ds_read_b_perm(s, j):
    c, h = j // 2, j % 2
    return f"ds_read_b128 %[b{s}_{j}], %[rb{s}{h}] offset:{c * 4096}"


def ktile_v2(first=False, bar_a=20, wait_at=104, dma_at=None, rd_early=None, rd_late=None, vm_extra_mode=None):
    """Schedule v2 (the hipBLASLt MT256x256x64 loop's placement, read from its gfx950 code object):
    the k-step-1 fragments of THIS K-tile are read first (MFMA 0..15), one barrier frees the buffer, the
    16 LDS-DMA pieces of K-tile t + 2 spread over the rest of the K-tile, and the wait for K-tile t + 1
    sits as LATE as possible (MFMA wait_at), right before the next K-tile's k-step-0 reads at the end.
    Returns (lines, n_dma_before_wait).  vm_extra_mode: None, or (mode operand, extra stores) -> the
    wait allows that many more operations when the mode SGPR is 2 (first K-tile after an epilogue)."""
    if dma_at is None:
        dma_at = [bar_a + 1 + 6 * q for q in range(16)]
    if rd_early is None:
        rd_early = list(range(16))
    if rd_late is None:
        rd_late = [wait_at + 2 + q for q in range(16)]
    assert max(rd_late) < 128 and max(dma_at) < 128 and min(dma_at) > bar_a > max(rd_early)
    order = [(i, j) for i in range(8) for j in range(8)]
    reads = read_order()
    dmas = [dma("a", j) for j in range(8)] + [dma("b", j) for j in range(8)]
    at = {n: q for q, n in enumerate(dma_at)}
    re_ = {n: q for q, n in enumerate(rd_early)}
    rl = {n: q for q, n in enumerate(rd_late)}
    n_before = sum(1 for n in dma_at if n < wait_at)
    lines = []
    for n in range(128):
        ks, (i, j) = n // 64, order[n % 64]
        if n == bar_a:
            lines += ["s_waitcnt lgkmcnt(0)", "s_barrier"]
        if n == wait_at:
            if vm_extra_mode:
                lines += ["s_cmp_eq_u32 %[mode], 2", "s_cbranch_scc1 LW%=_", f"s_waitcnt vmcnt({n_before})",
                          "s_branch LV%=_", "LW%=_:", f"s_waitcnt vmcnt({min(63, n_before + vm_extra_mode)})", "LV%=_:"]
            else:
                lines.append(f"s_waitcnt vmcnt({n_before})")
            lines += ["s_barrier", "v_xor_b32 %[ra0], 0x10000, %[ra0]", "v_xor_b32 %[rb00], 0x10000, %[rb00]",
                      "v_xor_b32 %[rb01], 0x10000, %[rb01]"]
        if n in re_:
            kind, idx = reads[re_[n]]
            lines.append(ds_read(1, kind, idx, "ra1") if kind == "a" else ds_read_b_perm(1, idx))
        if n in rl:
            kind, idx = reads[rl[n]]
            lines.append(ds_read(0, kind, idx, "ra0") if kind == "a" else ds_read_b_perm(0, idx))
        if n in at:
            lines += dmas[at[n]]
        lines.append(mfma(ks, i, j, zero_c=first and ks == 0))
    lines += ["v_xor_b32 %[ra1], 0x10000, %[ra1]", "v_xor_b32 %[rb10], 0x10000, %[rb10]",
              "v_xor_b32 %[rb11], 0x10000, %[rb11]", "s_waitcnt lgkmcnt(0)"]
    return lines


def ktile_v2_modes(vm_extra=32, **kw):
    """v2 with the persistent kernel's mode branch (see ktile_nt_modes): k-step 0 zero-accumulates in
    modes 1 / 2; the late wait allows vm_extra more operations in mode 2."""
    normal = ktile_v2(vm_extra_mode=vm_extra, **kw)
    first = ktile_v2(first=True, vm_extra_mode=vm_extra, **kw)
    # the bodies differ only in the k-step-0 MFMAs (index < the first k-step-1 MFMA line)
    k1n = next(k for k, l in enumerate(normal) if l.startswith("v_mfma") and "b1_" in l)
    k1f = next(k for k, l in enumerate(first) if l.startswith("v_mfma") and "b1_" in l)
    assert normal[k1n:] == first[k1f:]
    lines = ["s_nop 4", "s_cmp_eq_u32 %[mode], 0", "s_cbranch_scc0 LF%=_"]
    lines += normal[:k1n] + ["s_branch LJ%=_", "LF%=_:"] + first[:k1f] + ["LJ%=_:"] + normal[k1n:]
    return lines


def ktile_nt_modes(vm_extra=32, **kw):
    """The persistent kernel's K-tile: ONE asm statement for every position in the stream (one call
    site keeps the compiler from shuffling the accumulators between sites), branching on the SGPR
    operand mode: 0 = a continuing K-tile; 1 = the first K-tile of the workgroup's first tile; 2 = the
    first K-tile of a later tile (k-step 0 accumulates onto 0, and barrier B leaves the previous tile's
    vm_extra epilogue stores in flight).  Both k-step-0 bodies issue the same DMAs, so the counts match."""
    normal = ktile_nt(**kw)
    first = ktile_nt(first=True, **kw)
    i64n = next(k for k, l in enumerate(normal) if l.startswith("s_waitcnt vmcnt("))
    i64f = next(k for k, l in enumerate(first) if l.startswith("s_waitcnt vmcnt("))
    assert normal[i64n + 1:] == first[i64f + 1:]
    before_b = int(normal[i64n].split("(")[1].rstrip(")"))
    assert normal[0] == first[0] == "s_nop 4"
    lines = ["s_nop 4", "s_cmp_eq_u32 %[mode], 0", "s_cbranch_scc0 LF%=_"]
    lines += normal[1:i64n] + ["s_branch LJ%=_", "LF%=_:"] + first[1:i64f] + ["LJ%=_:"]
    lines += ["s_cmp_eq_u32 %[mode], 2", "s_cbranch_scc1 LW%=_", f"s_waitcnt vmcnt({before_b})", "s_branch LV%=_",
              "LW%=_:", f"s_waitcnt vmcnt({min(63, before_b + vm_extra)})", "LV%=_:"]
    lines += normal[i64n + 1:]
    return lines


# schedule variants (gemm4.hip template parameter SCHED; diagnostic ones selected by MFT_G4_DIAG)
VARIANTS = {
    "NT": dict(),                                                  # 0: the product schedule
    "NT_NODMA": dict(with_dma=False),                              # 1: no LDS-DMA (wrong output)
    "NT_FAST_SPREAD4": dict(read_gap=1, bar_a=20, dma_at=[21 + 4 * q for q in range(16)]),  # 2
    "NT_FAST_SPREAD2": dict(read_gap=1, bar_a=20, dma_at=[21 + 2 * q for q in range(16)]),  # 3
    "NT_SPREAD6": dict(read_gap=1, bar_a=20, dma_at=[22 + 6 * q for q in range(16)]),       # 4
    # persistent kernel: the first K-tile of a tile (after the previous tile's 32 / 64 epilogue stores)
    "NT_FIRST": dict(first=True),
    "NT_FIRST_S32": dict(first=True, vm_extra=32),
    "NT_FIRST_S64": dict(first=True, vm_extra=64),
}


def operands(modes=False):
    outs = [f'[c{i}{j}] "+a"(ACC[{i * 8 + j}])' for i in range(8) for j in range(8)]
    outs += [f'[a0_{i}] "+v"(FA0[{i}])' for i in range(8)] + [f'[b0_{j}] "+v"(FB0[{j}])' for j in range(8)]
    outs += [f'[a1_{i}] "=&v"(FA1[{i}])' for i in range(8)] + [f'[b1_{j}] "=&v"(FB1[{j}])' for j in range(8)]
    outs += ['[ra0] "+v"(RA0)', '[ra1] "+v"(RA1)', '[rb0] "+v"(RB0)', '[rb1] "+v"(RB1)']
    ins = [f'[oa{j}] "v"(OA[{j}])' for j in range(8)] + [f'[ob{j}] "v"(OB[{j}])' for j in range(8)]
    ins += ['[srda] "s"(SRDA)', '[srdb] "s"(SRDB)', '[koff] "s"(KOFF)', '[ldsm] "s"(LDSM)']
    if modes:
        ins.append('[mode] "s"(MODE)')
    return outs, ins


def emit(name, lines, modes=False):
    outs, ins = operands(modes)
    body = "".join(f'    "{l}\\n"  \\\n' for l in lines)
    extra = ", MODE" if modes else ""
    return (f"#define {name}(ACC, FA0, FB0, FA1, FB1, RA0, RA1, RB0, RB1, OA, OB, SRDA, SRDB, KOFF, LDSM{extra}) \\\n"
            f"  asm volatile(  \\\n{body}"
            f"    : {', '.join(outs)}  \\\n"
            f"    : {', '.join(ins)}  \\\n"
            f"    : \"memory\", \"scc\")\n")


FRAG_BASE = 128  # explicit-register form: fragment sets in v[128:255], accumulators in a[0:255]


def explicit(lines):
    """Rewrite the %[...] accumulator / fragment operands to literal registers (persistent kernel: no
    compiler-managed tuple operands, so no allocator shuffles them between statements)."""
    import re

    def acc(m):
        i, j = int(m.group(1)), int(m.group(2))
        b = 4 * (8 * i + j)
        return f"a[{b}:{b + 3}]"

    def frag(m):
        kind, st, idx = m.group(1), int(m.group(2)), int(m.group(3))
        b = FRAG_BASE + 64 * st + (0 if kind == "a" else 32) + 4 * idx
        return f"v[{b}:{b + 3}]"

    out = []
    for l in lines:
        l = re.sub(r"%\[c(\d)(\d)\]", acc, l)
        l = re.sub(r"%\[([ab])([01])_(\d)\]", frag, l)
        out.append(l)
    return out


def clobbers(fragments=True):
    regs = ([f"v{r}" for r in range(FRAG_BASE, 256)] if fragments else []) + [f"a{r}" for r in range(256)]
    return ", ".join(f'"{r}"' for r in regs)


def emit_explicit(name, lines, modes=True):
    """Literal registers: the accumulators a[0:255] and both fragment sets v[128:255] are clobbers of
    every statement, so the compiler keeps none of its own values there across a statement.  What
    crosses statements in them (set 0 between K-tiles, the accumulators into the epilogue) is read
    back by statements too (gemm4.hip: accr, and the kernel keeps no compiler value live there)."""
    ins = ['[ra0] "+v"(RA0)', '[ra1] "+v"(RA1)', '[rb00] "+v"(RB[0])', '[rb01] "+v"(RB[1])', '[rb10] "+v"(RB[2])',
           '[rb11] "+v"(RB[3])']
    ins_only = [f'[oa{j}] "v"(OA[{j}])' for j in range(8)] + [f'[ob{j}] "v"(OB[{j}])' for j in range(8)]
    ins_only += ['[srda] "s"(SRDA)', '[srdb] "s"(SRDB)', '[koff] "s"(KOFF)', '[ldsm] "s"(LDSM)']
    if modes:
        ins_only.append('[mode] "s"(MODE)')
    body = "".join(f'    "{l}\\n"  \\\n' for l in explicit(lines))
    return (f"#define {name}(RA0, RA1, RB, OA, OB, SRDA, SRDB, KOFF, LDSM, MODE) \\\n"
            f"  asm volatile(  \\\n{body}"
            f"    : {', '.join(ins)}  \\\n"
            f"    : {', '.join(ins_only)}  \\\n"
            '    : "memory", "scc", ' + clobbers() + ")\n")


def set0_read_explicit():
    """The first k-step's fragments of a tile (buffer of RA0 / RB) into set 0, waited for."""
    lines = [f"ds_read_b128 v[{FRAG_BASE + 4 * i}:{FRAG_BASE + 4 * i + 3}], %[ra0] offset:{i * 2048}" for i in range(8)]
    lines += [f"ds_read_b128 v[{FRAG_BASE + 32 + 4 * j}:{FRAG_BASE + 32 + 4 * j + 3}], %[rb0{j % 2}] offset:{(j // 2) * 4096}"
              for j in range(8)]
    lines.append("s_waitcnt lgkmcnt(0)")
    body = "".join(f'    "{l}\\n"  \\\n' for l in lines)
    regs = ", ".join(f'"v{r}"' for r in range(FRAG_BASE, FRAG_BASE + 64))
    return (f"#define GEMM4_SET0_READ_X(RA0, RB) \\\n  asm volatile(  \\\n{body}"
            '    :  \\\n    : [ra0] "v"(RA0), [rb00] "v"(RB[0]), [rb01] "v"(RB[1])  \\\n    : "memory", ' + regs + ")\n")


def ktile_tn(bar_a=32, wait_at=96, late_at=97, late_per=2, early_per=1, dma_at0=None, dma_step=4):
    """TN K-tile (weight gradient dW = dy^T x, both operands token-major): the LDS images are [64 k][256
    columns] (512-B rows, 16-B chunks XOR-swizzled on bits 1..3 by the row), and a fragment is TWO
    ds_read_b64_tr_b16 (rows k .. k + 3 and k + 4 .. k + 7 of a 16-lane group -> the lane's column, CDNA
    HIP guide T10) into the halves of its 4-VGPR register.  The swizzle makes fragment i's address
    base + 32 (i ^ t) with a per-lane t, so every fragment has its own address VGPR (%[ra{i}] / %[rb{j}],
    16 in all); the k-step (16384 B) and the half (2048 B) are immediate offsets, and one v_xor of all 16
    moves them to the other buffer.  Schedule (per K-tile t, buffer cur = t & 1; the product placement
    TN_VARIANTS["GEMM4_KTILE_TN_X"]):
        MFMA 0..15    32 reads of (t, ks 1) -> set 1 (two per MFMA)
        MFMA 16       lgkmcnt(0) + barrier: buffer cur is free
        MFMA 17..107  16 LDS-DMA pieces of K-tile t + 2 -> buffer cur (one per 6 MFMAs)
        MFMA 112      vmcnt(16) + barrier: K-tile t + 1 landed; the 16 addresses -> buffer cur ^ 1
        MFMA 112..127 32 reads of (t + 1, ks 0) -> set 0 (two per MFMA); lgkmcnt(0) at the end"""
    order = [(i, j) for i in range(8) for j in range(8)]
    reads = []
    for kind, idx in read_order():
        reads += [(kind, idx, 0), (kind, idx, 1)]

    def rd(s, ks, r):
        kind, idx, h = r
        b = FRAG_BASE + 64 * s + (0 if kind == "a" else 32) + 4 * idx + 2 * h
        return f"ds_read_b64_tr_b16 v[{b}:{b + 1}], %[r{kind}{idx}] offset:{ks * 16384 + h * 2048}"

    def dma_tn(kind, j):
        off = (0 if kind == "a" else 32768) + j * 4096
        return [f"s_add_u32 m0, %[ldsm], {off}", "s_nop 0",
                f"buffer_load_dwordx4 %[o{kind}{j}], %[srd{kind}], %[koff{kind}] offen lds"]

    dmas = [dma_tn("a", j) for j in range(8)] + [dma_tn("b", j) for j in range(8)]
    d0 = bar_a + 1 if dma_at0 is None else dma_at0
    dma_at = {d0 + dma_step * q: q for q in range(16)}
    assert max(dma_at) < wait_at and min(dma_at) > bar_a and 32 // early_per <= bar_a
    late = {}
    for q in range(32):
        late.setdefault(late_at + q // late_per, []).append(q)
    assert max(late) < 128
    lines = ["s_nop 4"]
    for n in range(128):
        ks, (i, j) = n // 64, order[n % 64]
        if n == bar_a:
            lines += ["s_waitcnt lgkmcnt(0)", "s_barrier"]
        if n == wait_at:
            lines += ["s_waitcnt vmcnt(16)", "s_barrier"]
            lines += [f"v_xor_b32 %[r{k}{x}], 0x10000, %[r{k}{x}]" for k in "ab" for x in range(8)]
        for q in range(n * early_per, (n + 1) * early_per):
            if q < 32:
                lines.append(rd(1, 1, reads[q]))
        for q in late.get(n, []):
            lines.append(rd(0, 0, reads[q]))
        if n in dma_at:
            lines += dmas[dma_at[n]]
        lines.append(mfma(ks, i, j))
    lines.append("s_waitcnt lgkmcnt(0)")
    return lines


# TN schedule variants (gemm4.hip gemm4_tn_kernel template SCHED, MFT_WGRAD_SCHED=0..2 for A/B)
TN_VARIANTS = {
    # 0 (product): k-step-1 reads two per MFMA (0..15), DMAs one per 6 MFMAs (17..107), the wait late (112),
    # the next k-step-0 reads two per MFMA -- the best of 7 placements measured (profiles/r6_wgrad_tn.txt)
    "GEMM4_KTILE_TN_X": dict(early_per=2, bar_a=16, dma_at0=17, dma_step=6, wait_at=112, late_at=112),
    "GEMM4_KTILE_TN_X1": dict(dma_step=5, wait_at=110, late_at=110),               # 1: reads one per MFMA
    "GEMM4_KTILE_TN_X2": dict(dma_step=4, wait_at=96, late_at=97),                 # 2: the first placement
}


def emit_tn(name, lines):
    ins = [f'[ra{i}] "+v"(RA[{i}])' for i in range(8)] + [f'[rb{j}] "+v"(RB[{j}])' for j in range(8)]
    ins_only = [f'[oa{j}] "v"(OA[{j}])' for j in range(8)] + [f'[ob{j}] "v"(OB[{j}])' for j in range(8)]
    ins_only += ['[srda] "s"(SRDA)', '[srdb] "s"(SRDB)', '[koffa] "s"(KOFFA)', '[koffb] "s"(KOFFB)', '[ldsm] "s"(LDSM)']
    body = "".join(f'    "{l}\\n"  \\\n' for l in explicit(lines))
    return (f"#define {name}(RA, RB, OA, OB, SRDA, SRDB, KOFFA, KOFFB, LDSM) \\\n"
            f"  asm volatile(  \\\n{body}"
            f"    : {', '.join(ins)}  \\\n"
            f"    : {', '.join(ins_only)}  \\\n"
            '    : "memory", "scc", ' + clobbers() + ")\n")


def tn_set0_read():
    """The first k-step's fragments (buffer of RA / RB, ks 0) into set 0, waited for."""
    lines = []
    for kind, idx in read_order():
        for h in range(2):
            b = FRAG_BASE + (0 if kind == "a" else 32) + 4 * idx + 2 * h
            lines.append(f"ds_read_b64_tr_b16 v[{b}:{b + 1}], %[r{kind}{idx}] offset:{h * 2048}")
    lines.append("s_waitcnt lgkmcnt(0)")
    body = "".join(f'    "{l}\\n"  \\\n' for l in lines)
    ins = [f'[ra{i}] "v"(RA[{i}])' for i in range(8)] + [f'[rb{j}] "v"(RB[{j}])' for j in range(8)]
    regs = ", ".join(f'"v{r}"' for r in range(FRAG_BASE, FRAG_BASE + 64))
    return (f"#define GEMM4_TN_SET0_READ_X(RA, RB) \\\n  asm volatile(  \\\n{body}"
            f"    :  \\\n    : {', '.join(ins)}  \\\n    : \"memory\", " + regs + ")\n")


def zero_acc():
    body = "".join(f'    "v_accvgpr_write_b32 a{r}, 0\\n"  \\\n' for r in range(256))
    return "#define GEMM4_ZERO_ACC_X() \\\n  asm volatile(  \\\n" + body + "    ::: " + clobbers(fragments=False) + ")\n"


def main():
    here = os.path.dirname(os.path.abspath(__file__))
    out = os.path.join(here, "gemm4_sched.h")
    with open(out, "w") as f:
        f.write("// GENERATED by gen_gemm4.py -- do not edit.  One K-tile of gemm4 (kernels/gemm4.hip) per schedule\n"
                "// variant: 128 MFMA, 32 ds_read_b128, 16 LDS-DMA pieces per wave.\n#pragma once\n\n")
        for name, kw in VARIANTS.items():
            lines = ktile_nt(**kw)
            n_mfma = sum(1 for l in lines if l.startswith("v_mfma"))
            n_rd = sum(1 for l in lines if l.startswith("ds_read"))
            n_dma = sum(1 for l in lines if l.startswith("buffer_load"))
            assert (n_mfma, n_rd) == (128, 32) and n_dma in (0, 16), (name, n_mfma, n_rd, n_dma)
            f.write(f"// {name}: {kw}\n")
            f.write(emit("GEMM4_KTILE_" + name, lines))
            f.write("\n")
        for S in (32, 40, 48, 64):  # stores per wave of the previous tile's epilogue: 32 / CE_FWD 40 / GEGLU_FWD 48 / 2 outputs 64
            lines = ktile_v2_modes(vm_extra=S)
            assert sum(1 for l in lines if l.startswith("v_mfma")) == 192
            n_dma = sum(1 for l in lines if l.startswith("buffer_load"))
            lf, lj = lines.index("LF%=_:"), lines.index("LJ%=_:")
            in_first = sum(1 for l in lines[lf:lj] if l.startswith("buffer_load"))
            assert n_dma - in_first == 16, (n_dma, in_first)  # one path issues exactly 16
            f.write(f"// V2_X{S}: schedule v2, literal registers, mode branch (persistent kernel)\n")
            f.write(emit_explicit(f"GEMM4_KTILE_V2_X{S}", lines))
            f.write("\n")

            if S in (40, 48):
                continue
            assert sum(1 for l in lines if l.startswith("v_mfma")) == 192
            f.write(f"// NT_P{S}: persistent K-tile, mode-branching (previous tile's epilogue: {S} stores per wave)\n")
            f.write(emit(f"GEMM4_KTILE_NT_P{S}", lines, modes=True))
            f.write("\n")
        f.write(set0_read_explicit())
        for name, kw in TN_VARIANTS.items():
            lines = ktile_tn(**kw)
            assert sum(1 for l in lines if l.startswith("v_mfma")) == 128
            assert sum(1 for l in lines if l.startswith("ds_read_b64_tr_b16")) == 64
            assert sum(1 for l in lines if l.startswith("buffer_load")) == 16
            f.write(f"\n// {name}: weight-gradient K-tile (token-major operands, transposed LDS reads), literal registers {kw}\n")
            f.write(emit_tn(name, lines))
            f.write("\n")
        f.write(tn_set0_read())
        f.write("\n")
        f.write(zero_acc())
    print(out)


if __name__ == "__main__":
    main()
