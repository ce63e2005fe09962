# C5 replay: what the board count mirror costs (timing only, results wrong):
# nomirror: the step kernel does not write it and the count reads one plane of it
F = "sl_bits128.hip"
VARIANTS = {
    "nomirror": [(F, """        if (MODE != SPAWN_PHILOX && me) {
#pragma unroll
            for (int s = 0; s < 4; s++)""", """        if (MODE != SPAWN_PHILOX && me && lane > 99) {
#pragma unroll
            for (int s = 0; s < 4; s++)"""),
                 (F, """                for (int q = 0; q < 2; q++) M[t][s][q] = me[t * 512 + (2 * s + q) * 64];""",
                  """                for (int q = 0; q < 2; q++) M[t][s][q] = s ? M[t][0][q] : me[t * 512 + (2 * s + q) * 64];""")],
}
