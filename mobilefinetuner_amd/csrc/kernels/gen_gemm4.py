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


def mfma(s, i, j):
    return f"v_mfma_f32_16x16x32_bf16 %[c{i}{j}], %[b{s}_{j}], %[a{s}_{i}], %[c{i}{j}]"


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


def ktile_nt(read_gap=READ_GAP, bar_a=BAR_A, dma_at=None, with_dma=True):
    """One K-tile: MFMA n = 0..127 (k-step n // 64).  dma_at[q] = the MFMA index (> bar_a) the q-th of
    the 16 LDS-DMA pieces precedes; the ones before MFMA 64 are left in flight by barrier B's vmcnt."""
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
            lines += [f"s_waitcnt vmcnt({before_b})", "s_barrier",
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
        lines.append(mfma(ks, i, j))
    lines += ["v_xor_b32 %[ra1], 0x10000, %[ra1]", "v_xor_b32 %[rb1], 0x10000, %[rb1]", "s_waitcnt lgkmcnt(0)"]
    return lines


# schedule variants (gemm4.hip template parameter SCHED; diagnostic ones selected by MFT_G4_DIAG)
VARIANTS = {
    "NT": dict(),                                                  # 0: the product schedule
    "NT_NODMA": dict(with_dma=False),                              # 1: no LDS-DMA (wrong output)
    "NT_FAST_SPREAD4": dict(read_gap=1, bar_a=20, dma_at=[21 + 4 * q for q in range(16)]),  # 2
    "NT_FAST_SPREAD2": dict(read_gap=1, bar_a=20, dma_at=[21 + 2 * q for q in range(16)]),  # 3
    "NT_SPREAD6": dict(read_gap=1, bar_a=20, dma_at=[22 + 6 * q for q in range(16)]),       # 4
}


def operands():
    outs = [f'[c{i}{j}] "+a"(ACC[{i * 8 + j}])' for i in range(8) for j in range(8)]
    outs += [f'[a0_{i}] "+v"(FA0[{i}])' for i in range(8)] + [f'[b0_{j}] "+v"(FB0[{j}])' for j in range(8)]
    outs += [f'[a1_{i}] "=&v"(FA1[{i}])' for i in range(8)] + [f'[b1_{j}] "=&v"(FB1[{j}])' for j in range(8)]
    outs += ['[ra0] "+v"(RA0)', '[ra1] "+v"(RA1)', '[rb0] "+v"(RB0)', '[rb1] "+v"(RB1)']
    ins = [f'[oa{j}] "v"(OA[{j}])' for j in range(8)] + [f'[ob{j}] "v"(OB[{j}])' for j in range(8)]
    ins += ['[srda] "s"(SRDA)', '[srdb] "s"(SRDB)', '[koff] "s"(KOFF)', '[ldsm] "s"(LDSM)']
    return outs, ins


def emit(name, lines):
    outs, ins = operands()
    body = "".join(f'    "{l}\\n"  \\\n' for l in lines)
    return (f"#define {name}(ACC, FA0, FB0, FA1, FB1, RA0, RA1, RB0, RB1, OA, OB, SRDA, SRDB, KOFF, LDSM) \\\n"
            f"  asm volatile(  \\\n{body}"
            f"    : {', '.join(outs)}  \\\n"
            f"    : {', '.join(ins)}  \\\n"
            f"    : \"memory\")\n")


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
    print(out)


if __name__ == "__main__":
    main()
