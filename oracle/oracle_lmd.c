/*
 * oracle_lmd.c -- TEST INFRASTRUCTURE ONLY (see roms_oracle.h).
 * LMD/KPP vertical mixing restatement (lmd_vmix.F, lmd_kpp.F): pending.
 */
#include <stdio.h>
#include "oracle_core.h"

void or_lmd_alloc(or_state *S) { (void)S; }
void or_lmd_vmix_impl(or_state *S, int tind) {
  (void)S; (void)tind;
  fprintf(stderr, "oracle: LMD/KPP not yet restated\n");
  abort();
}
