// ncio.cpp -- netCDF classic 64-bit-offset (CDF-2) writer/reader (ncio.h).
#include "ncio.h"

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstring>
#include <stdexcept>

namespace roms {
namespace nc {

namespace {

constexpr uint32_t kDimTag = 0x0A, kVarTag = 0x0B, kAttTag = 0x0C;

int type_size(int t) {
  switch (t) {
    case NC_BYTE: case NC_CHAR: return 1;
    case NC_SHORT: return 2;
    case NC_INT: case NC_FLOAT: return 4;
    case NC_DOUBLE: return 8;
    default: throw std::runtime_error("ncio: unsupported type");
  }
}
int64_t pad4(int64_t n) { return (n + 3) & ~int64_t(3); }

struct Out {
  std::vector<unsigned char> b;
  void u32(uint32_t v) { for (int s = 24; s >= 0; s -= 8) b.push_back((unsigned char)(v >> s)); }
  void u64(uint64_t v) { for (int s = 56; s >= 0; s -= 8) b.push_back((unsigned char)(v >> s)); }
  void bytes(const void* p, size_t n) {
    const unsigned char* c = (const unsigned char*)p;
    b.insert(b.end(), c, c + n);
    while (b.size() % 4) b.push_back(0);
  }
  void name(const std::string& s) { u32((uint32_t)s.size()); bytes(s.data(), s.size()); }
  void att(const Att& a) {
    name(a.name);
    u32((uint32_t)a.type);
    if (a.type == NC_CHAR) { u32((uint32_t)a.text.size()); bytes(a.text.data(), a.text.size()); }
    else if (a.type == NC_INT) {
      u32((uint32_t)a.ints.size());
      for (int v : a.ints) u32((uint32_t)v);
    } else if (a.type == NC_DOUBLE) {
      u32((uint32_t)a.dbls.size());
      for (double v : a.dbls) { uint64_t u; std::memcpy(&u, &v, 8); u64(u); }
    } else {
      throw std::runtime_error("ncio: unsupported attribute type");
    }
  }
  void atts(const std::vector<Att>& v) {
    if (v.empty()) { u32(0); u32(0); return; }
    u32(kAttTag); u32((uint32_t)v.size());
    for (const Att& a : v) att(a);
  }
};

struct In {
  const std::vector<unsigned char>& b;
  size_t p = 0;
  uint32_t u32() {
    if (p + 4 > b.size()) throw std::runtime_error("ncio: truncated header");
    uint32_t v = 0;
    for (int q = 0; q < 4; q++) v = (v << 8) | b[p++];
    return v;
  }
  uint64_t u64() { uint64_t hi = u32(); return (hi << 32) | u32(); }
  std::string str(size_t n) {
    if (p + n > b.size()) throw std::runtime_error("ncio: truncated header");
    std::string s((const char*)&b[p], n);
    p += (size_t)pad4((int64_t)n);
    return s;
  }
  std::string name() { return str(u32()); }
  std::vector<Att> atts() {
    std::vector<Att> v;
    const uint32_t tag = u32(), n = u32();
    if (tag == 0 && n == 0) return v;
    if (tag != kAttTag) throw std::runtime_error("ncio: bad attribute list");
    for (uint32_t q = 0; q < n; q++) {
      Att a;
      a.name = name();
      a.type = (int)u32();
      const uint32_t ne = u32();
      if (a.type == NC_CHAR) a.text = str(ne);
      else if (a.type == NC_INT) { for (uint32_t e = 0; e < ne; e++) a.ints.push_back((int)u32()); }
      else if (a.type == NC_DOUBLE) {
        for (uint32_t e = 0; e < ne; e++) { uint64_t u = u64(); double d; std::memcpy(&d, &u, 8); a.dbls.push_back(d); }
      } else {
        p += (size_t)pad4((int64_t)ne * type_size(a.type));   // kept out of the model: skipped
      }
      v.push_back(a);
    }
    return v;
  }
};

void swap_copy(unsigned char* dst, const unsigned char* src, int64_t n, int w) {
  for (int64_t e = 0; e < n; e++)
    for (int q = 0; q < w; q++) dst[e * w + q] = src[e * w + (w - 1 - q)];
}

void pwrite_all(int fd, const void* p, size_t n, int64_t off) {
  const char* c = (const char*)p;
  while (n > 0) {
    const ssize_t r = ::pwrite(fd, c, n, (off_t)off);
    if (r <= 0) throw std::runtime_error("ncio: write failed");
    c += r; n -= (size_t)r; off += r;
  }
}
void pread_all(int fd, void* p, size_t n, int64_t off) {
  char* c = (char*)p;
  while (n > 0) {
    const ssize_t r = ::pread(fd, c, n, (off_t)off);
    if (r <= 0) throw std::runtime_error("ncio: read past the end of the file");
    c += r; n -= (size_t)r; off += r;
  }
}

}  // namespace

int64_t Var::count() const { return vsize / type_size(type); }

int File::add_dim(const std::string& name, int64_t len) {
  const int q = find_dim(name);
  if (q >= 0) {
    if (dims[q].len != len) throw std::runtime_error("ncio: dimension " + name + " redefined with another length");
    return q;
  }
  dims.push_back(Dim{name, len});
  return (int)dims.size() - 1;
}
int File::find_dim(const std::string& name) const {
  for (size_t q = 0; q < dims.size(); q++)
    if (dims[q].name == name) return (int)q;
  return -1;
}
int File::add_var(const std::string& name, int type, const std::vector<int>& dimids, std::vector<Att> atts) {
  if (find_var(name) >= 0) throw std::runtime_error("ncio: variable " + name + " defined twice");
  Var v;
  v.name = name; v.type = type; v.dims = dimids; v.atts = std::move(atts);
  int64_t n = type_size(type);
  for (size_t q = 0; q < dimids.size(); q++) {
    const Dim& d = dims.at(dimids[q]);
    if (d.len == 0) {
      if (q != 0) throw std::runtime_error("ncio: the record dimension must come first");
      v.is_rec = true;
    } else {
      n *= d.len;
    }
  }
  v.vsize = pad4(n);
  vars.push_back(v);
  return (int)vars.size() - 1;
}
int File::find_var(const std::string& name) const {
  for (size_t q = 0; q < vars.size(); q++)
    if (vars[q].name == name) return (int)q;
  return -1;
}
const Att* File::find_gatt(const std::string& name) const {
  for (const Att& a : gatts)
    if (a.name == name) return &a;
  return nullptr;
}

std::vector<unsigned char> File::header() const {
  Out o;
  const unsigned char magic[4] = {'C', 'D', 'F', 2};
  o.b.insert(o.b.end(), magic, magic + 4);
  o.u32((uint32_t)numrecs);
  if (dims.empty()) { o.u32(0); o.u32(0); }
  else {
    o.u32(kDimTag); o.u32((uint32_t)dims.size());
    for (const Dim& d : dims) { o.name(d.name); o.u32((uint32_t)d.len); }
  }
  o.atts(gatts);
  if (vars.empty()) { o.u32(0); o.u32(0); }
  else {
    o.u32(kVarTag); o.u32((uint32_t)vars.size());
    for (const Var& v : vars) {
      o.name(v.name);
      o.u32((uint32_t)v.dims.size());
      for (int d : v.dims) o.u32((uint32_t)d);
      o.atts(v.atts);
      o.u32((uint32_t)v.type);
      o.u32(v.vsize > 0xFFFFFFFFll ? 0xFFFFFFFFu : (uint32_t)v.vsize);
      o.u64((uint64_t)v.begin);
    }
  }
  return o.b;
}

void File::layout(int64_t header_bytes) {
  int64_t off = pad4(header_bytes);
  for (Var& v : vars)
    if (!v.is_rec) { v.begin = off; off += v.vsize; }
  recsize_ = 0;
  for (Var& v : vars)
    if (v.is_rec) { v.begin = off + recsize_; recsize_ += v.vsize; }
}

void File::create(const std::string& path) {
  close();
  numrecs = 0;
  layout((int64_t)header().size());   // begin offsets do not change the header length
  fd_ = ::open(path.c_str(), O_RDWR | O_CREAT | O_TRUNC, 0644);
  if (fd_ < 0) throw std::runtime_error("ncio: cannot create " + path);
  writable_ = true;
  const std::vector<unsigned char> h = header();
  pwrite_all(fd_, h.data(), h.size(), 0);
  // fixed variables are zero-filled up to the first record
  int64_t end = pad4((int64_t)h.size());
  for (const Var& v : vars)
    if (!v.is_rec && v.begin + v.vsize > end) end = v.begin + v.vsize;
  if (::ftruncate(fd_, (off_t)end) != 0) throw std::runtime_error("ncio: cannot size " + path);
}

void File::parse(const std::vector<unsigned char>& h) {
  In in{h};
  if (h.size() < 8 || h[0] != 'C' || h[1] != 'D' || h[2] != 'F') throw std::runtime_error("ncio: not a netCDF classic file");
  const int version = h[3];
  if (version != 1 && version != 2) throw std::runtime_error("ncio: unsupported netCDF classic version");
  in.p = 4;
  numrecs = in.u32();
  dims.clear(); gatts.clear(); vars.clear();
  uint32_t tag = in.u32(), n = in.u32();
  if (tag == kDimTag)
    for (uint32_t q = 0; q < n; q++) { Dim d; d.name = in.name(); d.len = in.u32(); dims.push_back(d); }
  gatts = in.atts();
  tag = in.u32(); n = in.u32();
  if (tag == kVarTag) {
    for (uint32_t q = 0; q < n; q++) {
      Var v;
      v.name = in.name();
      const uint32_t nd = in.u32();
      for (uint32_t e = 0; e < nd; e++) v.dims.push_back((int)in.u32());
      v.atts = in.atts();
      v.type = (int)in.u32();
      v.vsize = in.u32();
      v.begin = version == 2 ? (int64_t)in.u64() : (int64_t)in.u32();
      v.is_rec = !v.dims.empty() && dims.at(v.dims[0]).len == 0;
      int64_t cnt = type_size(v.type);   // exact size (vsize may be clamped for huge variables)
      for (size_t e = v.is_rec ? 1 : 0; e < v.dims.size(); e++) cnt *= dims.at(v.dims[e]).len;
      v.vsize = pad4(cnt);
      vars.push_back(v);
    }
  }
  recsize_ = 0;
  for (const Var& v : vars)
    if (v.is_rec) recsize_ += v.vsize;
}

void File::open(const std::string& path, bool writable) {
  close();
  fd_ = ::open(path.c_str(), writable ? O_RDWR : O_RDONLY);
  if (fd_ < 0) throw std::runtime_error("ncio: cannot open " + path);
  writable_ = writable;
  struct stat st;
  if (fstat(fd_, &st) != 0) throw std::runtime_error("ncio: cannot stat " + path);
  // the header is read in growing chunks until it parses
  size_t n = 1 << 16;
  for (;;) {
    const size_t m = n < (size_t)st.st_size ? n : (size_t)st.st_size;
    std::vector<unsigned char> h(m);
    pread_all(fd_, h.data(), m, 0);
    try {
      parse(h);
      return;
    } catch (const std::runtime_error& e) {
      if (m == (size_t)st.st_size || std::string(e.what()).find("truncated") == std::string::npos) throw;
      n *= 4;
    }
  }
}

void File::close() {
  if (fd_ >= 0) {
    if (writable_ && dirty_) {
      unsigned char b[4] = {(unsigned char)(numrecs >> 24), (unsigned char)(numrecs >> 16), (unsigned char)(numrecs >> 8),
                            (unsigned char)numrecs};
      pwrite_all(fd_, b, 4, 4);
    }
    ::close(fd_);
  }
  fd_ = -1;
  dirty_ = false;
}
File::~File() {
  try { close(); } catch (...) {}
}

int64_t File::offset(const Var& v, int64_t rec) const { return v.is_rec ? v.begin + rec * recsize_ : v.begin; }

template <class T>
static void put_any(int fd, const Var& v, int64_t off, const T* data) {
  const int64_t n = v.count();
  std::vector<unsigned char> buf((size_t)v.vsize, 0);
  swap_copy(buf.data(), (const unsigned char*)data, n, (int)sizeof(T));
  pwrite_all(fd, buf.data(), buf.size(), off);
}
template <class T>
static void get_any(int fd, const Var& v, int64_t off, T* data) {
  const int64_t n = v.count();
  std::vector<unsigned char> buf((size_t)(n * (int64_t)sizeof(T)));
  pread_all(fd, buf.data(), buf.size(), off);
  swap_copy((unsigned char*)data, buf.data(), n, (int)sizeof(T));
}

void File::put_double(int varid, int64_t rec, const double* data) {
  const Var& v = vars.at(varid);
  if (v.type != NC_DOUBLE) throw std::runtime_error("ncio: " + v.name + " is not double");
  put_any(fd_, v, offset(v, rec), data);
  if (v.is_rec && rec + 1 > numrecs) { numrecs = rec + 1; dirty_ = true; }
}
void File::put_int(int varid, int64_t rec, const int* data) {
  const Var& v = vars.at(varid);
  if (v.type != NC_INT) throw std::runtime_error("ncio: " + v.name + " is not int");
  put_any(fd_, v, offset(v, rec), data);
  if (v.is_rec && rec + 1 > numrecs) { numrecs = rec + 1; dirty_ = true; }
}
void File::get_double(int varid, int64_t rec, double* data) const {
  const Var& v = vars.at(varid);
  if (v.type != NC_DOUBLE) throw std::runtime_error("ncio: " + v.name + " is not double");
  if (v.is_rec && (rec < 0 || rec >= numrecs)) throw std::runtime_error("ncio: record out of range for " + v.name);
  get_any(fd_, v, offset(v, rec), data);
}
void File::get_int(int varid, int64_t rec, int* data) const {
  const Var& v = vars.at(varid);
  if (v.type != NC_INT) throw std::runtime_error("ncio: " + v.name + " is not int");
  if (v.is_rec && (rec < 0 || rec >= numrecs)) throw std::runtime_error("ncio: record out of range for " + v.name);
  get_any(fd_, v, offset(v, rec), data);
}

}  // namespace nc
}  // namespace roms
