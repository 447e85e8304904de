// The MT19937 runtime direct jump rows D_1 .. D_2048 (L = 17 * 2^14 words),
// computed at build time by csrc/gen_mt_rt_rows.cpp (lib/mt_rt_rows14.bin,
// 5.1 MB) and checked at first use (csrc/host_gf2poly.cpp, embedded_rows).
        .section .rodata.dn_mt_rt_rows14,"a",@progbits
        .balign 64
        .globl  dn_mt_rt_rows14_blob
        .hidden dn_mt_rt_rows14_blob
dn_mt_rt_rows14_blob:
        .incbin "lib/mt_rt_rows14.bin"
        .globl  dn_mt_rt_rows14_blob_end
        .hidden dn_mt_rt_rows14_blob_end
dn_mt_rt_rows14_blob_end:
        .section .note.GNU-stack,"",@progbits
