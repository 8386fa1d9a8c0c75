"""LDS bank model of dec10_kernel's compact tile (C0 floats per decode_0 input position, 16-byte
chunk c4 at c4 ^ key(position)): extra cycles per instruction for decode_0's operand reads
(ds_read_b128, one position per lane, 16-lane groups, bank = dword mod 64) and decode_1's
result stores (ds_write_b128, 8-lane groups, bank = dword mod 32), for candidate keys.
    python tools/lds/dec10_banks.py"""
RG = [[0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27], [4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31]]
RG += [[g + 32 for g in gr] for gr in RG]
C0, TA, TW = 32, 4, 32
LCY, NCH = TW + 1, C0 // 4


def cost(key):
    addr = lambda pos, c4: pos * C0 + 4 * (c4 ^ key(pos))
    rd = n = 0
    for w in range(2 * TA * TW // 64):
        for dy in (-1, 0):
            for dx in (-1, 0):
                for c4 in range(NCH):
                    a = {}
                    for l in range(64):
                        tid = 64 * w + l
                        r, c = tid // TW, tid % TW
                        a[l] = addr((r + 1 + dy) * LCY + c + 1 + dx, c4)
                    for gr in RG:
                        b = {}
                        for l in gr:
                            b.setdefault((a[l] % 64) // 4, set()).add(a[l])
                        rd += max(len(v) for v in b.values()) - 1
                    n += 1
    wr = m = 0
    for wave in range(TA):
        for p in range(4):
            py, px = p >> 1, p & 1
            for nb in range(C0 // 16):
                a = {}
                for l in range(64):
                    li, lg = l & 15, l >> 4
                    a[l] = addr((1 + 2 * wave + py) * LCY + 1 + 2 * li + px, nb * 4 + lg)
                for g0 in range(0, 64, 8):
                    b = {}
                    for l in range(g0, g0 + 8):
                        b.setdefault((a[l] % 32) // 4, set()).add(a[l])
                    wr += max(len(v) for v in b.values()) - 1
                m += 1
    return round(rd / n, 2), round(wr / m, 2)


if __name__ == "__main__":
    for name, k in [("(pos / 2) % 8 (shipped)", lambda p: (p // 2) % 8), ("pos % 8", lambda p: p % 8),
                    ("(pos >> 1) % 8 ^ (pos & 1) * 4", lambda p: ((p >> 1) % 8) ^ ((p & 1) * 4)),
                    ("(pos + pos // 8) % 8", lambda p: (p + p // 8) % 8), ("(pos/2 + pos/16) % 8", lambda p: (p // 2 + p // 16) % 8),
                    ("(pos ^ pos>>3) % 8", lambda p: (p ^ (p >> 3)) % 8), ("(pos/2 ^ pos/16) % 8", lambda p: ((p // 2) ^ (p // 16)) % 8)]:
        print(f"{name:34s} decode_0 reads / decode_1 stores: {cost(k)}")
