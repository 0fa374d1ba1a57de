// Host-side driver for tests/test_ncio.py: exercises the library's netCDF
// classic (CDF-2) writer/reader (ucla-roms_amd/csrc/ncio.cpp) without a GPU.
//   ncio_roundtrip write PATH        -- a file with fixed + record variables, 3 records,
//                                       then a 4th appended after reopening
//   ncio_roundtrip read PATH VAR REC -- prints the record as %.17g values, one per line
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../ucla-roms_amd/csrc/ncio.h"

using namespace roms::nc;

static double val(int rec, long idx) { return rec * 1000.0 + idx + 0.25; }

int main(int argc, char** argv) {
  if (argc >= 3 && !strcmp(argv[1], "write")) {
    File f;
    const int dt = f.add_dim("time", 0), dx = f.add_dim("xi_rho", 5), dy = f.add_dim("eta_rho", 3);
    const int dz = f.add_dim("s_rho", 2), da = f.add_dim("auxil", 6);
    f.gatts.push_back(Att::i("partition", {1, 4, 7, 9}));
    f.gatts.push_back(Att::str("title", "ncio round trip"));
    f.gatts.push_back(Att::d("dt", {300.0}));
    const int vh = f.add_var("h", NC_DOUBLE, {dy, dx}, {Att::str("units", "meter")});
    const int vt = f.add_var("ocean_time", NC_DOUBLE, {dt}, {Att::str("units", "second")});
    const int vs = f.add_var("time_step", NC_INT, {dt, da});
    const int vz = f.add_var("zeta", NC_DOUBLE, {dt, dy, dx}, {Att::str("long_name", "free-surface elevation")});
    const int vu = f.add_var("u", NC_DOUBLE, {dt, dz, dy, dx});
    f.create(argv[2]);
    std::vector<double> h(15), z(15), u(30);
    for (int q = 0; q < 15; q++) h[q] = 100.0 + q;
    f.put_double(vh, 0, h.data());
    auto rec = [&](File& F, int r) {
      const double tm = 300.0 * r;
      F.put_double(F.find_var("ocean_time"), r, &tm);
      const int ts[6] = {r + 1, r + 1, r + 1, 0, 0, 0};
      F.put_int(F.find_var("time_step"), r, ts);
      for (int q = 0; q < 15; q++) z[q] = val(r, q);
      for (int q = 0; q < 30; q++) u[q] = -val(r, q);
      F.put_double(F.find_var("zeta"), r, z.data());
      F.put_double(F.find_var("u"), r, u.data());
    };
    (void)vt; (void)vs; (void)vz; (void)vu;
    for (int r = 0; r < 3; r++) rec(f, r);
    f.close();
    File g;
    g.open(argv[2], true);   // append a 4th record, as wrt_restart_file reopens its file
    rec(g, 3);
    g.close();
    return 0;
  }
  if (argc >= 5 && !strcmp(argv[1], "read")) {
    File f;
    f.open(argv[2], false);
    const int v = f.find_var(argv[3]);
    if (v < 0) { fprintf(stderr, "no variable %s\n", argv[3]); return 2; }
    const long rec = atol(argv[4]);
    const int64_t n = f.vars[v].count();
    if (f.vars[v].type == NC_INT) {
      std::vector<int> a(n);
      f.get_int(v, rec, a.data());
      for (int64_t q = 0; q < n; q++) printf("%d\n", a[q]);
    } else {
      std::vector<double> a(n);
      f.get_double(v, rec, a.data());
      for (int64_t q = 0; q < n; q++) printf("%.17g\n", a[q]);
    }
    printf("numrecs %lld\n", (long long)f.numrecs);
    return 0;
  }
  fprintf(stderr, "usage: ncio_roundtrip write PATH | read PATH VAR REC\n");
  return 1;
}
