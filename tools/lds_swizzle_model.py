"""LDS bank-conflict model of the passes' LDS accesses (MI355X_MICROARCH.md, LDS table):
ds_read_b64 is serviced as 2 groups of 32 lanes over 64 banks; ds_write_b64 and each access of
ds_read2_b64 / ds_read2st64_b64 / ds_write2_b64 as 4 groups of 16 lanes over 32 banks; each
extra distinct address on a busy bank adds one cycle.
Prints the LDS-array cycles per block-wide access pattern for candidate tile swizzles of the row
passes (tile_pos<32, 8>: element (line, r) at line * 8 + (r ^ s(line))), and the extra cycles of
k_col2's stage regions (col2_stage_write / col2_stage_store, hbx_passes.hip) for the r03 and r04
row placements under both read models -- the compiler emits ds_read2st64_b64 for the stage reads
at N = 1024, where r03's placement cost 8 extra cycles per read (rocprofv3: 67.1 M
SQ_LDS_BANK_CONFLICT cycles per 128-job launch)."""


def cycles(idxs, kind):
    if kind == "r64":
        groups, mod = [range(0, 32), range(32, 64)], 32
    else:
        groups, mod = [range(i * 16, (i + 1) * 16) for i in range(4)], 16
    tot = 0
    for g in groups:
        banks = {}
        for lane in g:
            a = idxs[lane]
            if a is None:
                continue
            banks.setdefault(a % mod, set()).add(a)
        tot += max((len(v) for v in banks.values()), default=0)
    return tot


SWIZZLES = {
    "q": lambda line: ((line & 31) >> 2) & 7,
    "q^b1": lambda line: (((line & 31) >> 2) ^ ((line >> 1) & 1)) & 7,
    "q^5b1": lambda line: (((line & 31) >> 2) ^ (((line >> 1) & 1) * 5)) & 7,
}


def patterns(s):
    def tp(line, r):
        return line * 8 + (r ^ s(line))

    res = {}

    def chunks(kind, fn):
        tot = 0
        for wave in range(4):
            for i in range(16):
                for half in (0, 1):
                    idx = []
                    for lane in range(64):
                        c = wave * 64 + lane + 256 * i
                        idx.append(fn(c // 4, (c % 4) * 2 + half))
                    tot += cycles(idx, kind)
        return tot

    res["rowinv_tile_write"] = chunks("w64", tp)
    res["rowfwd_store_read"] = chunks("r64", tp)

    def lanes(kind, nreg, line_of, valid=lambda t: True):
        tot = 0
        for wave in range(4):
            for k in range(nreg):
                idx = []
                for lane in range(64):
                    grp, t = wave * 2 + lane // 32, lane % 32
                    idx.append(tp(line_of(t, k), grp) if valid(t) else None)
                tot += cycles(idx, kind)
        return tot

    res["rowinv_tile_read"] = lanes("r64", 32, lambda t, k: t + 32 * k)
    res["rowfwd_tile_write"] = lanes("w64", 32, lambda t, k: (k % 2) * 512 + t + 32 * (k // 2))
    res["896_rowinv_read"] = lanes("r64", 32, lambda t, k: (t if t < 28 else 0) + 28 * k)
    res["896_rowfwd_write"] = lanes("w64", 32, lambda t, k: (k % 2) * 448 + t + 28 * (k // 2),
                                    valid=lambda t: t < 28)
    return res


def col2_pos_r03(R, sp, y):
    return sp * (64 // (256 // R)) + y


def col2_pos(R, sp, y):
    """hbx_passes.hip col2_pos<R> (r04)."""
    TL = 256 // R
    NSP = TL // 2
    HB = (16 // NSP).bit_length() - 1
    return sp * (32 // TL) + (y ^ (16 if ((y >> HB) & 1) and sp != NSP - 1 else 0))


def _extra(addrs, groups, mod):
    """Extra cycles: per lane group, the busiest bank's distinct addresses minus one (None = an
    inactive lane, EXEC off)."""
    tot = 0
    for g in groups:
        banks = {}
        for lane in g:
            a = addrs[lane]
            if a is not None:
                banks.setdefault(a % mod, set()).add(a)
        tot += max((len(v) for v in banks.values()), default=1) - 1
    return tot


def col2_stage_conflicts(R, pos):
    """Extra bank cycles per block-wide line set of k_col2's staging: (reads as 16-lane / 32-bank
    accesses, reads as 32-lane / 64-bank ds_read_b64, writes as 16-lane / 32-bank)."""
    G16 = [range(i * 16, (i + 1) * 16) for i in range(4)]
    G32 = [range(0, 32), range(32, 64)]
    TL = 256 // R
    NSP = TL // 2
    RS = max(R * (R + 1), R * R + 32)
    N = R * R
    rd16 = rd32 = wr = 0
    for wave in range(4):
        for i in range(N * TL // 2 // 256):
            for par in (0, 1):
                addrs = []
                for lane in range(64):
                    tid = wave * 64 + lane
                    sp, r, band0 = tid % NSP, (tid // NSP) % 16, tid // (8 * TL)
                    y = band0 * 16 + r + (32 // TL) * 16 * i
                    addrs.append(2 * ((2 * sp + par) * RS + pos(R, sp, y)))   # dword address
                rd16 += _extra(addrs, G16, 32)
                rd32 += _extra(addrs, G32, 64)
        for k2 in range(R):
            addrs = []
            for lane in range(64):
                g, t = (wave * 64 + lane) // R, lane % R
                addrs.append(2 * (g * RS + pos(R, g // 2, t + R * k2)))
            wr += _extra(addrs, G16, 32)
    return rd16, rd32, wr


def tile896_pos(kx, r):
    """hbx_passes896.hip tile896_pos (r04): k_rowfwd896's plane tile [kx < 448][8 rows]."""
    m = kx % 28
    return kx * 8 + (r ^ ((((m >> 2) & 7) ^ (((m >> 1) & 1) * 5)) & 7))


def tile_pos_32_8(line, r):
    """hbx_rowcol.hpp tile_pos<32, 8> (the r01-r03 k_rowfwd896 tile)."""
    return line * 8 + (r ^ ((((line & 31) >> 2) ^ (((line >> 1) & 1) * 5)) & 7))


def rowfwd896_tile_conflicts(pos):
    """Extra bank cycles of k_rowfwd896's plane tile per row block and plane: (lane-row writes
    kx = t + 28 k2 as ds_write_b64, 16-B chunk reads as ds_read_b64, the same as 16-lane reads)."""
    G16 = [range(i * 16, (i + 1) * 16) for i in range(4)]
    G32 = [range(0, 32), range(32, 64)]
    wr = rd64 = rd16 = 0
    for w in range(4):
        for k2 in range(16):
            addrs = []
            for lane in range(64):
                grp, t = w * 2 + lane // 32, lane % 32
                addrs.append(2 * pos(t + 28 * k2, grp) if t < 28 else None)
            wr += _extra(addrs, G16, 32)
        for i in range(7):
            for half in (0, 1):
                addrs = []
                for lane in range(64):
                    c = w * 64 + lane + 256 * i
                    addrs.append(2 * pos(c // 4, (c % 4) * 2 + half))
                rd64 += _extra(addrs, G32, 64)
                rd16 += _extra(addrs, G16, 32)
    return wr, rd64, rd16


def _wave(fn, rs=32 * 33):
    """float2 addresses of one wave (two 32-lane groups, regions rs apart) -> dword addresses."""
    out = []
    for lane in range(64):
        grp, t = lane // 32, lane % 32
        a = fn(t)
        out.append(None if a is None else 2 * (grp * rs + a))
    return out


def col896_conflicts(placement, b64_reads=0):
    """Extra LDS cycles per wave and line iteration of k_col896 (hbx_passes896.hip) from the two
    accesses with lane-dependent columns: fft896_ns_s2's transposed reads A'[tt][k1] (32 per
    transpose; the compiler emits ds_read2_b64 -- two 16-lane / 32-bank accesses -- for all but
    `b64_reads` of them, which go out as 32-lane / 64-bank ds_read_b64) and the H mirror's 15 reads.
    placement "r04": lanes 28..31 read column 0, H rows of 32; "r05": lanes 28..31 read columns
    28..31, H rows of 28 with lanes 28..31 on the four free banks."""
    G16 = [range(i * 16, (i + 1) * 16) for i in range(4)]
    G32 = [range(0, 32), range(32, 64)]
    if placement == "r04":
        k1 = lambda t: t if t < 28 else 0                                  # noqa: E731
        hm = lambda i, t: (31 - i) * 32 + ((28 - t) if 0 < t < 28 else 32)  # noqa: E731
    else:
        k1 = lambda t: t                                                   # noqa: E731
        hm = lambda i, t: (31 - i) * 28 + (28 if t == 0 else (28 - t) & 31)  # noqa: E731
    tr = sorted((_extra(_wave(lambda t: tt * 33 + k1(t)), G16, 32), tt) for tt in range(32))
    ex = sum(e for e, _ in tr[b64_reads:]) + sum(_extra(_wave(lambda t: tt * 33 + k1(t)), G32, 64)
                                                  for _, tt in tr[:b64_reads])
    ex += sum(_extra(_wave(lambda t: hm(i, t)), G16, 32) for i in range(17, 32))
    # the writers: H rows (16-lane ds_write2_b64) must stay conflict-free as well
    hw = (lambda i, t: i * 32 + t) if placement == "r04" else (lambda i, t: i * 28 + t if t < 28 else None)
    ex += sum(_extra(_wave(lambda t: hw(i, t)), G16, 32) for i in range(17))
    return ex


MIRROR_K1 = [0, 16, 1, 31, 3, 29, 4, 28, 5, 27, 7, 25, 8, 24, 12, 20,
             2, 30, 6, 26, 9, 23, 10, 22, 11, 21, 13, 19, 14, 18, 15, 17]   # hbx_fft.hpp kMirrorK1


def rowfwd32_tile_write_conflicts(k1_of):
    """Extra cycles of k_rowfwd32's lane-row plane-tile writes (tile_pos<32, 8> of line k1 + 32 k2,
    row = the lane group; 16-lane / 32-bank service of ds_write_b64 / write2st64) per row block
    and plane, for the lane -> k1 order `k1_of`."""
    G16 = [range(i * 16, (i + 1) * 16) for i in range(4)]
    ex = 0
    for w in range(4):
        for k2 in range(16):
            addrs = []
            for lane in range(64):
                grp, t = w * 2 + lane // 32, lane % 32
                addrs.append(2 * tile_pos_32_8(k1_of(t) + 32 * k2, grp))
            ex += _extra(addrs, G16, 32)
    return ex


def mirror_pair_order_ok(order=MIRROR_K1):
    """The r05 mirror-paired order: a permutation of 0..31, lanes 0 / 1 hold the self-mirrored
    k1 = 0 / 16, lanes (2m, 2m + 1) hold k1 and 32 - k1 (the partner is lane t ^ 1)."""
    if sorted(order) != list(range(32)) or order[:2] != [0, 16]:
        return False
    return all(order[2 * m] + order[2 * m + 1] == 32 for m in range(1, 16))


def tile_pos_16(line, r):
    """hbx_rowcol.hpp tile_pos<R, 16> (16-row tiles: the N = 256 k_rowfwd<16, 256>)."""
    return line * 16 + (r ^ (((line & 15) ^ ((line >> 4) & 1)) & 15))


B128_GROUPS = [[*range(0, 4), *range(12, 16), *range(20, 28)], [*range(4, 12), *range(16, 20), *range(28, 32)]]
B128_GROUPS += [[lane + 32 for lane in g] for g in B128_GROUPS]


def rowfwd16_chunk_read_conflicts(form, N=256, NT=256):
    """Extra LDS cycles per workgroup and row block of k_rowfwd<16, 256>'s plane-tile chunk reads
    (chunk c: line c / 8, rows r2 = 2 (c % 8) and r2 + 1): form "b64" = two ds_read_b64 (32-lane /
    64-bank groups; r04), "b128" = one ds_read_b128 of the aligned 16-B pair (r05)."""
    G32 = [range(0, 32), range(32, 64)]
    ex = 0
    for w in range(NT // 64):
        for i in range(N * 16 // 2 // NT):
            cs = [w * 64 + lane + NT * i for lane in range(64)]
            if form == "b64":
                for half in (0, 1):
                    addrs = [2 * tile_pos_16(c // 8, (c % 8) * 2 + half) for c in cs]
                    for g in G32:
                        used = {}
                        for lane in g:
                            for d in (0, 1):
                                used.setdefault((addrs[lane] + d) % 64, set()).add(addrs[lane] + d)
                        ex += max(len(v) for v in used.values()) - 1
            else:
                base = [2 * (tile_pos_16(c // 8, (c % 8) * 2) & ~1) for c in cs]
                for g in B128_GROUPS:
                    used = {}
                    for lane in g:
                        for d in range(4):
                            used.setdefault((base[lane] + d) % 64, set()).add(base[lane] + d)
                    ex += max(len(v) for v in used.values()) - 1
    return ex


if __name__ == "__main__":
    print("k_rowfwd<16> chunk reads: 2x ds_read_b64", rowfwd16_chunk_read_conflicts("b64"),
          "ds_read_b128", rowfwd16_chunk_read_conflicts("b128"))
    print("k_rowfwd32 tile writes: natural order", rowfwd32_tile_write_conflicts(lambda t: t),
          "mirror-paired", rowfwd32_tile_write_conflicts(lambda t: MIRROR_K1[t]), mirror_pair_order_ok())
    print("k_col896 extra LDS cycles per wave and line: r04", col896_conflicts("r04"), "r05", col896_conflicts("r05"))
    print("k_rowfwd896 tile (write, read_b64, read2): tile_pos<32, 8>", rowfwd896_tile_conflicts(tile_pos_32_8),
          "tile896_pos", rowfwd896_tile_conflicts(tile896_pos))
    for R in (32, 16):
        print(f"k_col2 R={R} stage (read2 16-lane, read_b64 32-lane, write): r03",
              col2_stage_conflicts(R, col2_pos_r03), "r04", col2_stage_conflicts(R, col2_pos))
    for name, s in SWIZZLES.items():
        print(f"{name:6s}", patterns(s))
