/*
 * ORACLE TEST INFRASTRUCTURE -- compiles the reference AGC (drivers/audio/audio_agc.c,
 * included from where it lies, nothing copied) and exposes its file-scope parameter block
 * `agc_wdsp` (audio_agc.c:24-94) read-only, so the product's host setup layer can be
 * pinned bit-for-bit against AudioAgc_SetupAgcWdsp (audio_agc.c:126-339).
 */
#include "audio_agc.c"

#include <stdio.h>
#include <string.h>
static unsigned oracle_bits(float f) { unsigned u; memcpy(&u, &f, 4); return u; }
void oracle_ref_agc_dump(void)
{
    const agc_variables_t* a = &agc_wdsp;
#define F(x) printf("  \"%s\": %u,\n", #x, oracle_bits(a->x))
#define I(x) printf("  \"%s\": %d,\n", #x, (int)a->x)
    printf("{\n");
    I(ring_buffsize); I(out_index); I(in_index); I(attack_buffsize); I(state); I(decay_type);
    I(hang_counter); I(remove_dc); I(n_tau);
    F(tau_attack); F(tau_decay); F(max_gain); F(var_gain); F(fixed_gain); F(max_input);
    F(out_targ); F(tau_fast_backaverage); F(tau_fast_decay); F(pop_ratio); F(tau_hang_backmult);
    F(hangtime); F(hang_thresh); F(tau_hang_decay); F(attack_mult); F(decay_mult);
    F(fast_decay_mult); F(fast_backmult); F(onemfast_backmult); F(out_target); F(min_volts);
    F(inv_out_target); F(slope_constant); F(inv_max_input); F(hang_level); F(hang_backmult);
    F(onemhang_backmult); F(hang_decay_mult); F(sample_rate);
    printf("  \"hang_enable\": %d, \"mode\": %d\n", agc_wdsp_conf.hang_enable, agc_wdsp_conf.mode);
    printf("}\n");
#undef F
#undef I
}
