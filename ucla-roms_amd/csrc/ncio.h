// ncio.h -- netCDF classic files, 64-bit-offset format (CDF-2), written and
// read natively (no netCDF library in this image).  The reference creates
// its history/restart files with nf90_create(..., nf90_netcdf4)
// (roms_read_write.F:1182) and reads them back with nf90_open/nf90_get_var
// (get_init.F), which accept every netCDF format, so a CDF-2 file carrying
// the reference's dimensions, variables and attributes is interchangeable
// with its own at the API level (ncdump, ncjoin, nf90_get_var).
//
// Layout (netCDF classic format specification): big-endian header
//   magic 'C','D','F',2 | numrecs | dim_list | gatt_list | var_list
// followed by the fixed-size variables, then the records (each record holds
// one slab of every record variable, in definition order).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace roms {
namespace nc {

enum Type { NC_BYTE = 1, NC_CHAR = 2, NC_SHORT = 3, NC_INT = 4, NC_FLOAT = 5, NC_DOUBLE = 6 };

struct Att {
  std::string name;
  int type = NC_CHAR;
  std::string text;             // NC_CHAR
  std::vector<int> ints;        // NC_INT
  std::vector<double> dbls;     // NC_DOUBLE
  static Att str(const std::string& n, const std::string& v) { Att a; a.name = n; a.type = NC_CHAR; a.text = v; return a; }
  static Att i(const std::string& n, std::vector<int> v) { Att a; a.name = n; a.type = NC_INT; a.ints = std::move(v); return a; }
  static Att d(const std::string& n, std::vector<double> v) { Att a; a.name = n; a.type = NC_DOUBLE; a.dbls = std::move(v); return a; }
};

struct Dim {
  std::string name;
  int64_t len = 0;   // 0: the record (unlimited) dimension
};

struct Var {
  std::string name;
  std::vector<int> dims;   // dimension ids, slowest first (C order; record dim first if present)
  std::vector<Att> atts;
  int type = NC_DOUBLE;
  int64_t vsize = 0;       // bytes of one record (record variable) or of the whole variable
  int64_t begin = 0;       // file offset of its data (first record)
  bool is_rec = false;
  int64_t count() const;   // elements per record (or in total)
};

// One open file.  Define mode: add_dim / add_var / gatts, then create().
// Data mode: put / get by variable and record.  Errors throw std::runtime_error.
class File {
 public:
  std::vector<Dim> dims;
  std::vector<Att> gatts;
  std::vector<Var> vars;
  int64_t numrecs = 0;

  int add_dim(const std::string& name, int64_t len);
  int find_dim(const std::string& name) const;
  int add_var(const std::string& name, int type, const std::vector<int>& dimids, std::vector<Att> atts = {});
  int find_var(const std::string& name) const;   // -1 if absent
  const Att* find_gatt(const std::string& name) const;

  void create(const std::string& path);   // writes the header (numrecs 0)
  void open(const std::string& path, bool writable);
  void close();                           // writes numrecs back if records were added
  ~File();

  // record `rec` (0-based) of a record variable, or the whole fixed variable (rec ignored)
  void put_double(int varid, int64_t rec, const double* data);
  void put_int(int varid, int64_t rec, const int* data);
  void get_double(int varid, int64_t rec, double* data) const;
  void get_int(int varid, int64_t rec, int* data) const;
  int64_t recsize() const { return recsize_; }

 private:
  int fd_ = -1;
  bool writable_ = false;
  bool dirty_ = false;
  int64_t recsize_ = 0;
  void layout(int64_t header_bytes);
  std::vector<unsigned char> header() const;
  void parse(const std::vector<unsigned char>& h);
  int64_t offset(const Var& v, int64_t rec) const;
};

}  // namespace nc
}  // namespace roms
