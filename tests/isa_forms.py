"""Packed-FP32 op_sel / neg instruction forms (mnemonic, modifiers as llvm-objdump prints them) that
tools/pk_probe.hip runs as kinds 16.. alone and beside another kernel's MFMA loop (tools/pk_probe.py).  The forms
cleared by that probe on the MI355X are listed in CLEARED (tests/test_isa_guard.py allows only those); KNOWN_BAD are the
forms it showed returning wrong lanes 48..63 beside MFMA work (round 5, profiles/r05i_pk_probe_isolation.log;
re-confirmed as controls in round 6)."""

PROBE_FORMS = {
    16: ('v_pk_fma_f32', 'op_sel_hi:[1,0,0]'),
    17: ('v_pk_fma_f32', 'op_sel_hi:[1,0,1]'),
    18: ('v_pk_fma_f32', 'op_sel_hi:[1,1,0]'),
    19: ('v_pk_fma_f32', 'op_sel_hi:[0,1,1]'),
    20: ('v_pk_fma_f32', 'op_sel_hi:[0,1,0]'),
    21: ('v_pk_fma_f32', 'op_sel:[1,0,0]'),
    22: ('v_pk_fma_f32', 'op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]'),
    23: ('v_pk_fma_f32', 'op_sel:[1,0,0] op_sel_hi:[0,0,1] neg_lo:[0,1,0]'),
    24: ('v_pk_fma_f32', 'op_sel:[1,0,0] op_sel_hi:[0,0,1] neg_hi:[0,1,0]'),
    25: ('v_pk_fma_f32', 'op_sel:[1,0,0] op_sel_hi:[1,0,1]'),
    26: ('v_pk_fma_f32', 'op_sel:[1,0,0] op_sel_hi:[1,1,0]'),
    27: ('v_pk_fma_f32', 'op_sel:[0,0,1] op_sel_hi:[1,1,0]'),
    28: ('v_pk_fma_f32', 'op_sel_hi:[1,1,0] neg_lo:[1,0,0] neg_hi:[1,0,0]'),
    29: ('v_pk_fma_f32', 'op_sel_hi:[1,0,1] neg_lo:[0,0,1] neg_hi:[0,0,1]'),
    30: ('v_pk_mul_f32', 'op_sel_hi:[1,0]'),
    31: ('v_pk_mul_f32', 'op_sel_hi:[0,1]'),
    32: ('v_pk_add_f32', 'op_sel_hi:[1,0] neg_lo:[0,1] neg_hi:[0,1]'),
    33: ('v_pk_add_f32', ''),
    34: ('v_pk_add_f32', 'neg_hi:[0,1]'),
    35: ('v_pk_add_f32', 'neg_lo:[0,1]'),
    36: ('v_pk_add_f32', 'neg_lo:[0,1] neg_hi:[0,1]'),
    37: ('v_pk_add_f32', 'neg_lo:[1,1] neg_hi:[1,1]'),
    38: ('v_pk_fma_f32', ''),
    39: ('v_pk_fma_f32', 'neg_lo:[0,0,1] neg_hi:[0,0,1]'),
    40: ('v_pk_mul_f32', ''),
    41: ('v_pk_add_f32', 'op_sel_hi:[1,0]'),   # round 6: conv_dects.hip
}

# cleared on the MI355X (profiles/r06a_pk_probe_forms.log): every kind 16..40 gave 0 of 8 differing runs beside the
# MFMA loop, while the known-bad controls (kinds 5, 7) differed in 8 of 8, lanes 48..63
CLEARED = set(PROBE_FORMS.values())   # kind 41: profiles/r06b_pk_probe_form41.log

KNOWN_BAD = {("v_pk_add_f32", "op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]"), ("v_pk_add_f32", "op_sel:[0,1] op_sel_hi:[1,0]")}
