# C3 with fused packed views: where the view's extra time goes (timing only, the views
# written are incomplete -- never for parity).  o_full: as shipped; o_nogather: no view
# gather/stores (board rows still put into LDS, exits moved); o_noput: neither the LDS
# board nor the gather (the planes-12-14 goal colours, scores and transposes remain).
F = "sl_bits.hip"
GATHER = """        for (int i = lane; i < nv; i += 64) {
            o[i] = cells[lds_cell_idx((ty + r) & (N - 1), (tx + c) & (N - 1))];"""
NOGATHER = """        for (int i = lane; i < nv && lfx.obs_vh > 1000; i += 64) {
            o[i] = cells[lds_cell_idx((ty + r) & (N - 1), (tx + c) & (N - 1))];"""
PUT = """            lds_put_board(buf, lane, PB);      // the start board in buf has been read out"""
OBS_CALL = """        write_obs(buf, fx, fl, b, lane);"""
VARIANTS = {
    "o_full": [],
    "o_nogather": [(F, GATHER, NOGATHER)],
    "o_noput": [(F, PUT, "            if (kernarg().fx.obs_vh > 1000) lds_put_board(buf, lane, PB);"),
                (F, OBS_CALL, "        if (kernarg().fx.obs_vh > 1000) write_obs(buf, fx, fl, b, lane);")],
}
