#!/usr/bin/env python3
"""Write a phase-timing copy of a step-kernel source (for tools/phase_timing.py):
s_memtime stamps at the phase boundaries of step_env, every 64th env's wave
emitting them, plus the sl_debug_phase_times export.  Build the copy with
-DSL_BITS_TIMING=1.

usage: mk_timing.py in_sl_bits.hip out.hip
"""
import sys

MACROS = r'''// phase timing (tuning builds only): s_memtime stamps of every 64th env's wave,
// read back with sl_debug_phase_times
#ifndef SL_BITS_TIMING
#define SL_BITS_TIMING 0
#endif
#if SL_BITS_TIMING
__device__ unsigned long long g_sl_phase[1024][10];
#define SL_TM_DECL unsigned long long sl_tm[10]
#define SL_TM(k) do { __builtin_amdgcn_sched_barrier(0); sl_tm[k] = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0); } while (0)
#define SL_TM_EMIT                                                                  \
    if ((b & 63) == 0 && lane == 0)                                                 \
        for (int k = 0; k < 10; k++) g_sl_phase[(b >> 6) & 1023][k] = sl_tm[k]
#else
#define SL_TM_DECL
#define SL_TM(k)
#define SL_TM_EMIT
#endif
'''
EXPORT = r'''
#if SL_BITS_TIMING
extern "C" int sl_debug_phase_times(unsigned long long *host) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_sl_phase), sizeof(g_sl_phase)) == hipSuccess
               ? 0 : -1;
}
#endif
'''


def main(src, dst):
    s = open(src).read()
    s = s.replace('#ifndef SL_BITS_ABL\n', MACROS + '#ifndef SL_BITS_ABL\n', 1)
    k = s.index('void step_env(')

    def before(sub, mark):
        nonlocal s
        p = s.index(sub, k)
        s = s[:p] + mark + '\n' + s[p:]

    def after(sub, mark):
        nonlocal s
        p = s.index(sub, k) + len(sub)
        s = s[:p] + '\n' + mark + s[p:]

    before('    const u32 V = load_record(', '    SL_TM_DECL;\n    SL_TM(0);')
    before('    SpawnCtx sc;\n', '    SL_TM(1);')
    before('    // ---- board: from LDS', '    SL_TM(2);')
    after('    wait_vm();\n', '    SL_TM(3);')
    before('    u32 PB[32];\n    read_pairs', '    SL_TM(4);')
    before('    // ---- scores over the new board', '    SL_TM(5);')
    before('    // ---- write back the changed rows', '    SL_TM(6);')
    before('    int reset = 0;\n', '    SL_TM(7);')
    after('    reset = __builtin_amdgcn_readfirstlane(reset);', '    SL_TM(8);')
    tail = '''        reinterpret_cast<int32_t *>(fx.scratch + 2 * st.B)[i] = (int32_t)b;
    }
}
'''
    assert tail in s
    s = s.replace(tail, tail[:-2] + '    SL_TM(9);\n    SL_TM_EMIT;\n}\n', 1)
    s += EXPORT
    open(dst, 'w').write(s)


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2])
