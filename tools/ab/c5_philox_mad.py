# C5: the Philox round's two 32x32 multiplies as one 64-bit product each (hi and lo from
# one v_mad_u64_u32) instead of a v_mul_hi_u32 + v_mul_lo_u32 pair
F = "sl_device.h"
OLD = """        uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
        uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;"""
NEW = """        const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;"""
VARIANTS = {"mad": [(F, OLD, NEW)]}
