

def test_lds_swizzle_conflict_free():
    """The LDS XOR swizzles of the MFMA GEMMs are bank-conflict-free for their fragment reads: every
    lane group of a ds_read_b128 (CDNA4 services it as 4 groups of 16 lanes, {0-3,12-15,20-27},
    {4-11,16-19,28-31}, {32-35,44-47,52-59}, {36-43,48-51,60-63}; 16 lanes x 16 B = the 64 four-byte banks)
    hits 16 distinct 16-byte slots of the 256-B bank row. qgemm.hip a_lds_off (512-B rows, row = lane & 15,
    chunk = 8*(lane >> 4) + ks) and qmm.hip qmm_a_off (128-B rows, row = i*32 + (lane & 31),
    chunk = 2*s + (lane >> 5))."""
    groups = [[*range(0, 4), *range(12, 16), *range(20, 28)], [*range(4, 12), *range(16, 20), *range(28, 32)],
              [*range(32, 36), *range(44, 48), *range(52, 60)], [*range(36, 44), *range(48, 52), *range(60, 64)]]
    assert sorted(sum(groups, [])) == list(range(64))
    def qgemm_off(r, c):
        rr = r & 15
        return r * 512 + ((c ^ (rr ^ ((rr + 4) & 8))) << 4)

    def qmm_off(r, c):
        return r * 128 + ((c ^ ((r >> 1) & 7)) << 4)

    for ks in range(8):
        for lanes in groups:
            slots = {(qgemm_off(l & 15, 8 * (l >> 4) + ks) % 256) // 16 for l in lanes}
            assert len(slots) == 16, (ks, lanes)
    for i in range(4):
        for s in range(4):
            for lanes in groups:
                slots = {(qmm_off(i * 32 + (l & 31), 2 * s + (l >> 5)) % 256) // 16 for l in lanes}
                assert len(slots) == 16, (i, s, lanes)
