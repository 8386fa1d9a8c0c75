"""LDS bank model of enc01_kernel's layer-0 operand gathers (ds_read_b32: lanes 0-31 and 32-63
are the two groups, bank = dword mod 32; MI355X_MICROARCH.md §LDS) for the RGB plane pitch
RGBP: extra cycles per wave-instruction, averaged over the 7 k-steps and both column planes.
    python tools/lds/enc01_banks.py"""
QJ = 17


def gathers(R0, RGBP):
    tot = n = 0
    for plane in range(2):
        for t in range(7):
            for half in range(2):
                banks = {}
                for l in range(32 * half, 32 * half + 32):
                    lg, li = l >> 4, l & 15
                    k = 4 * t + lg
                    if k >= 27:
                        k = 0  # the zero weight row reads offset 0
                    tap, c = k // 3, k % 3
                    ky, kx = tap // 3, tap % 3
                    q = 2 * plane + kx
                    a = c * RGBP + ky * 4 * QJ + (q & 3) * QJ + (q >> 2) + li
                    banks.setdefault(a % 32, set()).add(a)
                tot += max(len(v) for v in banks.values()) - 1
            n += 1
    return tot / n


if __name__ == "__main__":
    for th1 in (2, 4, 8):
        R0 = 4 * th1 + 3
        base = R0 * 4 * QJ
        for pad in range(0, 32, 4):
            print(f"TH1 {th1}: RGBP {base + pad:5d} (+{pad:2d}, mod 32 = {(base + pad) % 32:2d}): "
                  f"{gathers(R0, base + pad):.2f} extra cycles per gather")


def layout_cost(R0, RP4, RGBP):
    """(layer-0 gather extra cycles per instruction, staging-write extra cycles per instruction)
    for RGB rows RP4 floats apart (4 column planes of QJ) and channel planes RGBP apart."""
    g = 0.0
    n = 0
    for plane in range(2):
        for t in range(7):
            for half in range(2):
                banks = {}
                for l in range(32 * half, 32 * half + 32):
                    lg, li = l >> 4, l & 15
                    k = 4 * t + lg
                    if k >= 27:
                        k = 0
                    tap, c = k // 3, k % 3
                    ky, kx = tap // 3, tap % 3
                    q = 2 * plane + kx
                    a = c * RGBP + ky * RP4 + (q & 3) * QJ + (q >> 2) + li
                    banks.setdefault(a % 32, set()).add(a)
                g += max(len(v) for v in banks.values()) - 1
            n += 1
    w = 0.0
    m = 0
    NG = R0 * 17
    for i in range((NG + 255) // 256):
        for wave in range(4):
            for k in range(4):
                for c in range(3):
                    for half in range(2):
                        banks = {}
                        for l in range(32 * half, 32 * half + 32):
                            e = i * 256 + wave * 64 + l
                            if e >= NG:
                                continue
                            rr, gg = e // 17, e % 17
                            a = c * RGBP + rr * RP4 + k * QJ + gg
                            banks.setdefault(a % 32, set()).add(a)
                        if banks:
                            w += max(len(v) for v in banks.values()) - 1
                    m += 1
    return g / n, w / m


def search(th1=4):
    R0 = 4 * th1 + 3
    res = []
    for RP4 in range(68, 100):
        for RGBP in range(R0 * RP4, R0 * RP4 + 32):
            gc, wc = layout_cost(R0, RP4, RGBP)
            res.append((gc * 35 + wc * 24, gc, wc, RP4, RGBP, RGBP * 3 * 4))
    res.sort()
    return res[:8]


RG = [[0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27], [4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31]]
RG += [[g + 32 for g in gr] for gr in RG]


def t1_cost(C0, keyf, TH1=4):
    """Layer-1 tile (CMP form: C0 floats per slot, 16-byte chunk c4 at c4 ^ key(slot)):
    extra cycles per ds_read_b128 of load_b and per ds_write_b128 of put0."""
    NCH = C0 // 4
    LC1 = 34
    PS1 = C0
    KC1 = C0 // 16
    addr = lambda slot, c4: slot * PS1 + 4 * (c4 ^ keyf(slot, NCH))
    rr = n = 0
    WR = 4 if TH1 >= 4 else 2
    MB = TH1 // WR
    for wr in range(WR):
        for s in range(9 * KC1):
            tap, kc = s // KC1, s % KC1
            ky, kx = tap // 3, tap % 3
            for mb in range(MB):
                r = wr * MB + mb
                a = {}
                for l in range(64):
                    lg, li = l >> 4, l & 15
                    lp = (2 * r + ky) * LC1 + (kx & 1) * 17 + li + (kx >> 1)
                    a[l] = addr(lp, kc * 4 + lg)
                for gr in RG:
                    b = {}
                    for l in gr:
                        b.setdefault((a[l] % 64) // 4, set()).add(a[l])
                    rr += max(len(v) for v in b.values()) - 1
                n += 1
    ww = m = 0
    LR1 = 2 * TH1 + 1
    for wave in range(4):
        for jb in range(5):
            for nb in range(C0 // 16):
                slot0 = (wave >> 1) * LC1 + (wave & 1) * 17 + 2 * LC1 * jb
                a = {l: addr(slot0 + (l & 15), nb * 4 + (l >> 4)) for l in range(64)}
                for g0 in range(0, 64, 8):
                    b = {}
                    for l in range(g0, g0 + 8):
                        b.setdefault((a[l] % 32) // 4, set()).add(a[l])
                    ww += max(len(v) for v in b.values()) - 1
                m += 1
    return rr / n, ww / m


if __name__ == "__main__":
    for C0 in (16, 32):
        grp = 16 // (C0 // 4)
        print(C0, "key (slot / GRP) % NCH:", t1_cost(C0, lambda s, N: (s // grp) % N),
              " key slot % NCH:", t1_cost(C0, lambda s, N: s % N))
