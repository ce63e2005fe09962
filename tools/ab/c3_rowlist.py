# C3: changed board rows stored from the wave's LDS copy of the new board, compacted.
# Today a store instruction writes rows y and 32 + y together (even lanes hold rows
# 0-31, odd lanes 32-63), so a changed row drags its unchanged partner along (3 550 B
# written per env-step against ~1 590 B of changed rows).  Here the
# exact changed rows (the rule's change masks ORed per half -- DPP over same-parity
# lanes -- plus the rows the action edited) are listed in LDS by rank, and each store
# instruction writes 8 whole rows, 8 lanes x 16 B a row, from the LDS board.
F = "sl_bits.hip"
HELPER = """
// Per-half OR: bit y of the result is set when any lane of this lane's parity (rows
// 32 (lane & 1) + y) has it -- quad xor 2, then two row rotations keep the parity
__device__ __forceinline__ uint64_t changed_rows64(u32 cl) {
    u32 x = cl | dpp<0x4E>(cl);           // quad_perm [2,3,0,1]
    x |= dpp<0x124>(x);                   // row_ror:4
    x |= dpp<0x128>(x);                   // row_ror:8
    const u32 lo = (u32)__builtin_amdgcn_readlane((int)x, 0) | (u32)__builtin_amdgcn_readlane((int)x, 16) |
                   (u32)__builtin_amdgcn_readlane((int)x, 32) | (u32)__builtin_amdgcn_readlane((int)x, 48);
    const u32 hi = (u32)__builtin_amdgcn_readlane((int)x, 1) | (u32)__builtin_amdgcn_readlane((int)x, 17) |
                   (u32)__builtin_amdgcn_readlane((int)x, 33) | (u32)__builtin_amdgcn_readlane((int)x, 49);
    return ((uint64_t)hi << 32) | lo;
}

// The rows of M (bit r = row r) stored from the LDS board (lds_put_board's layout:
// chunk c of row r at chunk (c + 4 (r >> 5)) & 7), ANDed with `keep`: slot s = lane >> 3
// of each store instruction takes the s-th listed row, lane & 7 its 16-byte chunk.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void store_rows(lds_u32 *buf, uint8_t *rowlist, u32 *gb0, uint64_t M,
                                           u32 keep, int lane) {
    typedef __attribute__((address_space(3))) uint8_t lds_u8;
    typedef __attribute__((address_space(3))) u32x4 lds_u32x4;
    lds_u8 *rl = (lds_u8 *)rowlist;
    if ((M >> lane) & 1ull) rl[lanes_below(M)] = (uint8_t)lane;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const int n = __builtin_popcountll(M);
    const int c = lane & 7;
    for (int s = lane >> 3; s < n; s += 8) {
        const int row = rl[s];
        u32x4 v = *(const lds_u32x4 *)(buf + row * 32 + (((c + 4 * (row >> 5)) & 7) << 2));
        v &= keep;
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(gb0) + row * 8 + c);
    }
}
"""
R = [
    (F, """typedef __attribute__((address_space(3))) uint16_t lds_u16;
""", """typedef __attribute__((address_space(3))) uint16_t lds_u16;
""" + HELPER),
    (F, """                                         uint16_t *vm, const int32_t *__restrict__ actions,""",
        """                                         uint16_t *vm, uint8_t *rowlist,
                                         const int32_t *__restrict__ actions,"""),
    (F, """        if (VIEW && !hi) {
            // planes 12-14 hold the goal colours: the store masks them out again
            if (rb) {
#pragma unroll
                for (int y = 0; y < 32; y++)
                    if ((rb >> y) & 1u) gb[y * 32] = PB[y] & 0x8FFF8FFFu;
            }
            lds_put_board(buf, lane, PB);      // the start board in buf has been read out
        } else if (rb) {
#pragma unroll
            for (int y = 0; y < 32; y++)
                if ((rb >> y) & 1u) __builtin_nontemporal_store(PB[y], &gb[y * 32]);
        }""", """        uint64_t M = 0ull;
        if (rb) {
            M = changed_rows64(cb[0] | cb[1]);
#pragma unroll
            for (int k = 0; k < 4; k++)
                if (k < ne) M |= 1ull << (eidx[k] >> 6);
        }
        u32 *gb0 = reinterpret_cast<u32 *>(st.board + off);
        if (VIEW && !hi) {
            lds_put_board(buf, lane, PB);      // the start board in buf has been read out
            // planes 12-14 hold the goal colours: the store masks them out again
            if (rb) store_rows(buf, rowlist, gb0, M, 0x8FFF8FFFu, lane);
        } else if (rb) {
            lds_put_board(buf, lane, PB);
            store_rows(buf, rowlist, gb0, M, 0xFFFFFFFFu, lane);
        }"""),
    (F, """    __shared__ __attribute__((aligned(16))) uint16_t vmask[OBS >= 2 ? sl::obs::kFusedChanCells : 2];""",
        """    __shared__ __attribute__((aligned(16))) uint16_t vmask[OBS >= 2 ? sl::obs::kFusedChanCells : 2];
    __shared__ uint8_t rowlist[64];        // changed rows by rank (store_rows)"""),
    (F, """    step_env<OBS, MODE>(ka.st, ka.a, ka.fx, b, lane, buf, vmask, ka.actions, ka.ctp, ka.ctc,""",
        """    step_env<OBS, MODE>(ka.st, ka.a, ka.fx, b, lane, buf, vmask, rowlist, ka.actions, ka.ctp, ka.ctc,"""),
]
VARIANTS = {"rl_base": [], "rl_list": R}
