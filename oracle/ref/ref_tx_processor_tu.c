/*
 * ORACLE TEST INFRASTRUCTURE -- compiles the reference's transmit processor for the x86 host.
 *
 * drivers/audio/tx_processor.c is included from where it lies under /root/reference (nothing
 * is copied); read-only accessors expose its file-static TX filter instances so the oracle
 * can dump the coefficients the firmware configured (TxProcessor_Set, tx_processor.c:72-120).
 */
#include "tx_processor.c"

const arm_iir_lattice_instance_f32* oracle_ref_tx_lattice(void) { return &IIR_TXFilter; }
const arm_biquad_casd_df1_inst_f32* oracle_ref_tx_biquad(void) { return &IIR_TX_biquad; }

/* fm_subaudible_tone_table (drivers/audio/fm_subaudible_tone_table.h, included by tx_processor.c) */
const float* oracle_ref_subaudible_table(int* n)
{
    *n = (int)(sizeof fm_subaudible_tone_table / sizeof fm_subaudible_tone_table[0]);
    return fm_subaudible_tone_table;
}
