# nontemporal cache policy on the 64x64 kernel's board DMA (global_load_lds aux)
VARIANTS = {
    "dma_base": [],
    "dma_nt": [("sl_bits.hip", """        __builtin_amdgcn_global_load_lds((const void *)(s + row * 128 + c * 16),
                                         (__attribute__((address_space(3))) void *)(buf + k * 256),
                                         16, 0, 0);""", """        __builtin_amdgcn_global_load_lds((const void *)(s + row * 128 + c * 16),
                                         (__attribute__((address_space(3))) void *)(buf + k * 256),
                                         16, 0, 2);""")],
}
