# C3: the 64x64 reset wave's rolled-level gathers as one dword load per row when the
# roll's column shift is even (both cells of the lane's pair in one aligned dword),
# two u16 loads otherwise
F = "sl_bits.hip"
OLD = """    auto rolled = [&](const uint16_t *lv, u32 D[32]) {
#pragma unroll
        for (int y = 0; y < 32; y++) {
            const int sr = ((32 * h + y - dy) & 63) * N;
            D[y] = (u32)lv[sr + c0] | ((u32)lv[sr + c1] << 16);
        }
    };"""
NEW = """    auto rolled = [&](const uint16_t *lv, u32 D[32]) {
        if (!(dx & 1)) {
            const u32 *lw = reinterpret_cast<const u32 *>(lv);
#pragma unroll
            for (int y = 0; y < 32; y++) D[y] = lw[(((32 * h + y - dy) & 63) * N + c0) >> 1];
        } else {
#pragma unroll
            for (int y = 0; y < 32; y++) {
                const int sr = ((32 * h + y - dy) & 63) * N;
                D[y] = (u32)lv[sr + c0] | ((u32)lv[sr + c1] << 16);
            }
        }
    };"""
VARIANTS = {"rdw": [(F, OLD, NEW)]}
