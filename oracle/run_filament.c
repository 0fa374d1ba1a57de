/* TEST INFRASTRUCTURE: runs the Filament benchmark case through the oracle and
 * prints the diag code_check lines (format of diag.F: I2,1x,4ES23.16). */
#include <stdio.h>
#include <stdlib.h>
#include "roms_oracle.h"
int main(int argc, char **argv) {
  or_cfg c = {0};
  c.LLm = 64; c.MMm = 64; c.N = 32; c.NT = 1;
  c.ew_periodic = 1; c.ns_periodic = 1;
  c.dt = 5.0; c.ndtfast = 60; c.theta_s = 6.0; c.theta_b = 2.0; c.hc = 25.0; c.rho0 = 1000.0;
  c.rdrg = 0.0; c.rdrg2 = 1.0e-3; c.Zob = 1.e-2; c.Tcoef = 0.20; c.T0 = 1.0; c.Scoef = 0.822; c.S0 = 1.0;
  c.sizex = 12.8e3; c.sizey = 3.2e3; c.diag_np_xi = 3; c.diag_np_eta = 2;
  int nsteps = argc > 1 ? atoi(argv[1]) : 20;
  or_state *S = or_create(&c);
  or_init(S);
  double n[4];
  or_norms(S, n);
  printf("%2d %23.16E %23.16E %23.16E %23.16E\n", or_iic(S), n[0], n[1], n[2], n[3]);
  for (int s = 0; s < nsteps; s++) {
    or_step(S);
    or_norms(S, n);
    printf("%2d %23.16E %23.16E %23.16E %23.16E\n", or_iic(S), n[0], n[1], n[2], n[3]);
  }
  printf("nfast=%d\n", or_nfast(S));
  return 0;
}
