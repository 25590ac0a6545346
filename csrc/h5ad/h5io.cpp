// Minimal native HDF5 object API (libhdf5 C API) for the h5ad on-disk format.
//
// The reference reads/writes AnnData .h5ad files through scanpy/anndata/h5py
// (cnmf.py:519,545,698; preprocess.py:242-243).  None of those are available here, so
// cnmf_torch_amd ships this small native layer and implements the AnnData layout
// (X dense/csr/csc, obs/var dataframes, obsm, categoricals) in Python on top of it
// (cnmf_torch_amd/utils/h5ad.py).  Row-range reads (hyperslabs) let large matrices be
// streamed in chunks instead of loaded whole.
#include <hdf5.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace py = pybind11;

namespace {

struct H5Err : std::runtime_error {
  using std::runtime_error::runtime_error;
};

inline hid_t chk(hid_t id, const std::string& what) {
  if (id < 0) throw H5Err("HDF5 error: " + what);
  return id;
}
inline void chk(herr_t e, const std::string& what, int) {
  if (e < 0) throw H5Err("HDF5 error: " + what);
}

// RAII holder for any hid_t with its matching close function.
struct Hid {
  hid_t id = -1;
  herr_t (*closer)(hid_t) = nullptr;
  Hid() = default;
  Hid(hid_t i, herr_t (*c)(hid_t)) : id(i), closer(c) {}
  Hid(const Hid&) = delete;
  Hid& operator=(const Hid&) = delete;
  Hid(Hid&& o) noexcept : id(o.id), closer(o.closer) { o.id = -1; }
  Hid& operator=(Hid&& o) noexcept {
    if (this != &o) {
      if (id >= 0 && closer) closer(id);
      id = o.id;
      closer = o.closer;
      o.id = -1;
    }
    return *this;
  }
  ~Hid() {
    if (id >= 0 && closer) closer(id);
  }
  operator hid_t() const { return id; }
};

hid_t native_type_for(const py::dtype& dt) {
  const char kind = dt.kind();
  const size_t sz = dt.itemsize();
  if (kind == 'f') {
    if (sz == 4) return H5T_NATIVE_FLOAT;
    if (sz == 8) return H5T_NATIVE_DOUBLE;
  } else if (kind == 'i') {
    if (sz == 1) return H5T_NATIVE_INT8;
    if (sz == 2) return H5T_NATIVE_INT16;
    if (sz == 4) return H5T_NATIVE_INT32;
    if (sz == 8) return H5T_NATIVE_INT64;
  } else if (kind == 'u') {
    if (sz == 1) return H5T_NATIVE_UINT8;
    if (sz == 2) return H5T_NATIVE_UINT16;
    if (sz == 4) return H5T_NATIVE_UINT32;
    if (sz == 8) return H5T_NATIVE_UINT64;
  }
  throw H5Err("unsupported numpy dtype for HDF5 write");
}

// h5py stores numpy bool as an int8 enum {FALSE=0, TRUE=1}; mirror it so files
// round-trip with h5py/anndata.
Hid make_bool_enum() {
  hid_t t = chk(H5Tenum_create(H5T_NATIVE_INT8), "enum create");
  int8_t v = 0;
  H5Tenum_insert(t, "FALSE", &v);
  v = 1;
  H5Tenum_insert(t, "TRUE", &v);
  return Hid(t, H5Tclose);
}

Hid make_vlen_str() {
  hid_t t = chk(H5Tcopy(H5T_C_S1), "str type");
  H5Tset_size(t, H5T_VARIABLE);
  H5Tset_cset(t, H5T_CSET_UTF8);
  return Hid(t, H5Tclose);
}

Hid lcpl_intermediate() {
  hid_t p = chk(H5Pcreate(H5P_LINK_CREATE), "lcpl");
  H5Pset_create_intermediate_group(p, 1);
  return Hid(p, H5Pclose);
}

std::vector<hsize_t> shape_of(const py::array& a) {
  std::vector<hsize_t> s;
  for (py::ssize_t i = 0; i < a.ndim(); ++i) s.push_back((hsize_t)a.shape(i));
  return s;
}

py::dtype dtype_for_h5(hid_t t) {
  const H5T_class_t cls = H5Tget_class(t);
  const size_t sz = H5Tget_size(t);
  if (cls == H5T_FLOAT) return sz == 4 ? py::dtype("float32") : py::dtype("float64");
  if (cls == H5T_INTEGER) {
    const bool sgn = H5Tget_sign(t) == H5T_SGN_2;
    switch (sz) {
      case 1: return sgn ? py::dtype("int8") : py::dtype("uint8");
      case 2: return sgn ? py::dtype("int16") : py::dtype("uint16");
      case 4: return sgn ? py::dtype("int32") : py::dtype("uint32");
      default: return sgn ? py::dtype("int64") : py::dtype("uint64");
    }
  }
  throw H5Err("unsupported HDF5 numeric type");
}

hid_t mem_type_for(const py::dtype& dt) { return native_type_for(dt); }

bool is_bool_enum(hid_t t) {
  if (H5Tget_class(t) != H5T_ENUM) return false;
  return H5Tget_nmembers(t) == 2 && H5Tget_size(t) == 1;
}

// Read `n` string elements of type `ftype` from a dataset/attribute reader.
template <class ReadFn>
py::list read_strings(hid_t ftype, hsize_t n, ReadFn reader) {
  py::list out;
  if (H5Tis_variable_str(ftype) > 0) {
    std::vector<char*> buf(n, nullptr);
    Hid mt = make_vlen_str();
    if (n == 0) return out;
    reader((hid_t)mt, (void*)buf.data());
    for (hsize_t i = 0; i < n; ++i) {
      out.append(py::str(buf[i] ? buf[i] : ""));
    }
    // reclaim with a simple dataspace of n elements
    Hid sp(H5Screate_simple(1, &n, nullptr), H5Sclose);
    if (n) H5Dvlen_reclaim(mt, sp, H5P_DEFAULT, buf.data());
  } else {
    const size_t sz = H5Tget_size(ftype);
    std::vector<char> buf(sz * (n ? n : 1) + 1, 0);
    hid_t mt = chk(H5Tcopy(H5T_C_S1), "fstr");
    H5Tset_size(mt, sz);
    Hid mth(mt, H5Tclose);
    if (n == 0) return out;
    reader(mt, (void*)buf.data());
    for (hsize_t i = 0; i < n; ++i) {
      const char* s = buf.data() + i * sz;
      size_t len = strnlen(s, sz);
      out.append(py::str(std::string(s, len)));
    }
  }
  return out;
}

py::object read_attr_obj(hid_t attr) {
  Hid ft(H5Aget_type(attr), H5Tclose);
  Hid sp(H5Aget_space(attr), H5Sclose);
  const int nd = H5Sget_simple_extent_ndims(sp);
  std::vector<hsize_t> dims(nd > 0 ? nd : 0);
  if (nd > 0) H5Sget_simple_extent_dims(sp, dims.data(), nullptr);
  hsize_t n = 1;
  for (auto d : dims) n *= d;
  const H5T_class_t cls = H5Tget_class(ft);
  if (cls == H5T_STRING) {
    py::list l = read_strings(ft, n, [&](hid_t mt, void* buf) {
      chk(H5Aread(attr, mt, buf), "attr read", 0);
    });
    if (nd == 0) return l[0];
    return l;
  }
  if (is_bool_enum(ft)) {
    std::vector<int8_t> b(n);
    Hid et = make_bool_enum();
    chk(H5Aread(attr, et, b.data()), "attr bool read", 0);
    if (nd == 0) return py::bool_(b[0] != 0);
    py::array_t<bool> out(std::vector<py::ssize_t>(dims.begin(), dims.end()));
    for (hsize_t i = 0; i < n; ++i) out.mutable_data()[i] = b[i] != 0;
    return out;
  }
  if (cls == H5T_INTEGER || cls == H5T_FLOAT) {
    py::dtype dt = dtype_for_h5(ft);
    std::vector<py::ssize_t> shp(dims.begin(), dims.end());
    py::array out(dt, shp);
    chk(H5Aread(attr, mem_type_for(dt), out.mutable_data()), "attr read", 0);
    if (nd == 0) return out[py::tuple()];
    return out;
  }
  return py::none();
}

void write_attr_impl(hid_t obj, const std::string& name, py::handle value) {
  if (H5Aexists(obj, name.c_str()) > 0) H5Adelete(obj, name.c_str());
  if (py::isinstance<py::str>(value)) {
    std::string s = value.cast<std::string>();
    Hid t = make_vlen_str();
    Hid sp(H5Screate(H5S_SCALAR), H5Sclose);
    Hid a(chk(H5Acreate2(obj, name.c_str(), t, sp, H5P_DEFAULT, H5P_DEFAULT), "attr create"),
          H5Aclose);
    const char* p = s.c_str();
    chk(H5Awrite(a, t, &p), "attr write", 0);
    return;
  }
  if (py::isinstance<py::bool_>(value)) {
    Hid t = make_bool_enum();
    Hid sp(H5Screate(H5S_SCALAR), H5Sclose);
    Hid a(chk(H5Acreate2(obj, name.c_str(), t, sp, H5P_DEFAULT, H5P_DEFAULT), "attr create"),
          H5Aclose);
    int8_t v = value.cast<bool>() ? 1 : 0;
    chk(H5Awrite(a, t, &v), "attr write", 0);
    return;
  }
  if (py::isinstance<py::list>(value) || py::isinstance<py::tuple>(value)) {
    py::sequence seq = value.cast<py::sequence>();
    bool all_str = true;
    for (auto it : seq)
      if (!py::isinstance<py::str>(it)) all_str = false;
    if (all_str) {
      std::vector<std::string> ss;
      for (auto it : seq) ss.push_back(it.cast<std::string>());
      std::vector<const char*> ps;
      for (auto& s : ss) ps.push_back(s.c_str());
      hsize_t n = ps.size();
      Hid t = make_vlen_str();
      Hid sp(H5Screate_simple(1, &n, nullptr), H5Sclose);
      Hid a(chk(H5Acreate2(obj, name.c_str(), t, sp, H5P_DEFAULT, H5P_DEFAULT), "attr create"),
            H5Aclose);
      if (n) chk(H5Awrite(a, t, ps.data()), "attr write", 0);
      return;
    }
    value = py::module_::import("numpy").attr("asarray")(value);
  }
  py::array arr = py::array::ensure(value, py::array::c_style | py::array::forcecast);
  if (!arr) throw H5Err("cannot convert attribute value for " + name);
  if (arr.dtype().kind() == 'b') {
    arr = arr.attr("astype")("int8");
  }
  hid_t mt = native_type_for(arr.dtype());
  Hid sp = arr.ndim() == 0
               ? Hid(H5Screate(H5S_SCALAR), H5Sclose)
               : Hid(H5Screate_simple(arr.ndim(), shape_of(arr).data(), nullptr), H5Sclose);
  Hid a(chk(H5Acreate2(obj, name.c_str(), mt, sp, H5P_DEFAULT, H5P_DEFAULT), "attr create"),
        H5Aclose);
  chk(H5Awrite(a, mt, arr.data()), "attr write", 0);
}

// Raw parallel I/O of a contiguous, unfiltered dataset (HDF5 stores its elements as
// plain bytes at one file offset): large numeric X matrices are read / written with
// pread / pwrite from several threads instead of one H5Dread / H5Dwrite stream
// (~2.7 GB/s single-threaded on the GPU box: 1.5 s for the 500k-cell float64 norm
// counts, profiles/r4d_harmony_*).  The library never touches those bytes: the
// datasets are allocated early with no fill, and the metadata stays HDF5's.
constexpr size_t kRawMinBytes = size_t(64) << 20;
constexpr size_t kRawPiece = size_t(32) << 20;

// (buffered writes to one file serialise on its inode lock: a few threads only keep the
// page-cache copy going while another waits; reads scale with threads)
int raw_threads(bool write) { return write ? 4 : 8; }

// pread / pwrite of [0, nbytes) of buf at file offset off, in pieces over threads
bool raw_io(const std::string& path, bool write, haddr_t off, char* buf, size_t nbytes) {
  const int fd = ::open(path.c_str(), write ? O_WRONLY : O_RDONLY);
  if (fd < 0) return false;
  const size_t npieces = (nbytes + kRawPiece - 1) / kRawPiece;
  const int nt = (int)std::min<size_t>((size_t)raw_threads(write), npieces);
  std::atomic<size_t> next{0};
  std::atomic<bool> ok{true};
  auto work = [&]() {
    for (size_t i = next++; i < npieces && ok; i = next++) {
      size_t a = i * kRawPiece;
      const size_t b = std::min(nbytes, a + kRawPiece);
      while (a < b) {
        const ssize_t r = write ? ::pwrite(fd, buf + a, b - a, (off_t)(off + a))
                                : ::pread(fd, buf + a, b - a, (off_t)(off + a));
        if (r <= 0) {
          ok = false;
          break;
        }
        a += (size_t)r;
      }
    }
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < nt; ++t) pool.emplace_back(work);
  work();
  for (auto& t : pool) t.join();
  const bool closed = ::close(fd) == 0;
  return ok && closed;
}

// file offset of a dataset whose bytes are raw-accessible as `mt` (contiguous layout, no
// filters / external storage, allocated, file type == memory type), else HADDR_UNDEF
haddr_t raw_offset(hid_t d, hid_t mt) {
  const char* e = getenv("CNMF_H5_RAW");          // "0": HDF5's own I/O only
  if (e && e[0] == '0') return HADDR_UNDEF;
  Hid dcpl(H5Dget_create_plist(d), H5Pclose);
  if (dcpl.id < 0 || H5Pget_layout(dcpl) != H5D_CONTIGUOUS) return HADDR_UNDEF;
  if (H5Pget_nfilters(dcpl) != 0 || H5Pget_external_count(dcpl) != 0) return HADDR_UNDEF;
  Hid ft(H5Dget_type(d), H5Tclose);
  if (ft.id < 0 || H5Tequal(ft, mt) <= 0) return HADDR_UNDEF;
  return H5Dget_offset(d);
}

class File {
 public:
  File(const std::string& path, const std::string& mode) : path_(path) {
    H5Eset_auto2(H5E_DEFAULT, nullptr, nullptr);  // errors become exceptions, not stderr spam
    if (mode == "r") {
      fid_ = H5Fopen(path.c_str(), H5F_ACC_RDONLY, H5P_DEFAULT);
    } else if (mode == "r+") {
      fid_ = H5Fopen(path.c_str(), H5F_ACC_RDWR, H5P_DEFAULT);
    } else if (mode == "w") {
      fid_ = H5Fcreate(path.c_str(), H5F_ACC_TRUNC, H5P_DEFAULT, H5P_DEFAULT);
    } else {
      throw H5Err("mode must be r, r+ or w");
    }
    if (fid_ < 0) throw H5Err("cannot open HDF5 file " + path + " (mode " + mode + ")");
  }
  ~File() { close(); }
  void close() {
    if (fid_ >= 0) {
      H5Fclose(fid_);
      fid_ = -1;
    }
  }
  hid_t fid() const {
    if (fid_ < 0) throw H5Err("file is closed");
    return fid_;
  }

  bool exists(const std::string& p) const {
    if (p == "/" || p.empty()) return true;
    // check every prefix so a missing intermediate group is not an error
    std::string acc;
    size_t pos = 0;
    while (pos != std::string::npos) {
      size_t nxt = p.find('/', pos + 1);
      acc = p.substr(0, nxt);
      if (!acc.empty() && acc != "/") {
        if (H5Lexists(fid(), acc.c_str(), H5P_DEFAULT) <= 0) return false;
      }
      pos = nxt;
    }
    return true;
  }

  std::string kind(const std::string& p) const {
    if (!exists(p)) return "missing";
    Hid o(H5Oopen(fid(), p.c_str(), H5P_DEFAULT), H5Oclose);
    if (o.id < 0) return "missing";
    H5I_type_t t = H5Iget_type(o);
    if (t == H5I_GROUP) return "group";
    if (t == H5I_DATASET) return "dataset";
    return "other";
  }

  std::vector<std::string> list(const std::string& p) const {
    Hid g(chk(H5Gopen2(fid(), p.c_str(), H5P_DEFAULT), "open group " + p), H5Gclose);
    H5G_info_t info;
    chk(H5Gget_info(g, &info), "group info", 0);
    std::vector<std::string> names;
    for (hsize_t i = 0; i < info.nlinks; ++i) {
      ssize_t len = H5Lget_name_by_idx(g, ".", H5_INDEX_NAME, H5_ITER_INC, i, nullptr, 0,
                                       H5P_DEFAULT);
      std::string s(len, '\0');
      H5Lget_name_by_idx(g, ".", H5_INDEX_NAME, H5_ITER_INC, i, &s[0], len + 1, H5P_DEFAULT);
      names.push_back(s);
    }
    return names;
  }

  void create_group(const std::string& p) {
    if (exists(p)) return;
    Hid l = lcpl_intermediate();
    Hid g(chk(H5Gcreate2(fid(), p.c_str(), l, H5P_DEFAULT, H5P_DEFAULT), "create group " + p),
          H5Gclose);
  }

  void write_array(const std::string& p, py::array value, int compression) {
    if (exists(p)) chk(H5Ldelete(fid(), p.c_str(), H5P_DEFAULT), "unlink " + p, 0);
    py::array arr = py::array::ensure(value, py::array::c_style);
    if (!arr) throw H5Err("array must be convertible to C-contiguous");
    const bool is_bool = arr.dtype().kind() == 'b';
    Hid booltype;
    hid_t ft, mt;
    if (is_bool) {
      booltype = make_bool_enum();
      ft = booltype;
      mt = booltype;
    } else {
      ft = mt = native_type_for(arr.dtype());
    }
    std::vector<hsize_t> dims = shape_of(arr);
    Hid sp = arr.ndim() == 0 ? Hid(H5Screate(H5S_SCALAR), H5Sclose)
                             : Hid(H5Screate_simple(arr.ndim(), dims.data(), nullptr), H5Sclose);
    Hid dcpl(H5Pcreate(H5P_DATASET_CREATE), H5Pclose);
    hsize_t total = 1;
    for (auto d : dims) total *= d;
    if (compression > 0 && arr.ndim() >= 1 && total > 0) {
      std::vector<hsize_t> chunk(dims);
      // ~1 MiB chunks along the leading axis
      hsize_t row = 1;
      for (size_t i = 1; i < dims.size(); ++i) row *= dims[i];
      hsize_t rows = std::max<hsize_t>(1, (1u << 20) / std::max<hsize_t>(1, row * arr.itemsize()));
      chunk[0] = std::min<hsize_t>(dims[0], rows);
      for (auto& c : chunk) c = std::max<hsize_t>(c, 1);
      H5Pset_chunk(dcpl, (int)chunk.size(), chunk.data());
      H5Pset_deflate(dcpl, compression);
    }
    const size_t nbytes = (size_t)total * (size_t)arr.itemsize();
    const bool raw = compression <= 0 && !is_bool && arr.ndim() >= 1 && nbytes >= kRawMinBytes;
    if (raw) {               // allocated now, never filled: the raw writes are its contents
      H5Pset_layout(dcpl, H5D_CONTIGUOUS);
      H5Pset_alloc_time(dcpl, H5D_ALLOC_TIME_EARLY);
      H5Pset_fill_time(dcpl, H5D_FILL_TIME_NEVER);
    }
    Hid l = lcpl_intermediate();
    Hid d(chk(H5Dcreate2(fid(), p.c_str(), ft, sp, l, dcpl, H5P_DEFAULT), "create dataset " + p),
          H5Dclose);
    if (raw) {
      const haddr_t off = raw_offset(d, mt);
      if (off != HADDR_UNDEF) {
        chk(H5Fflush(fid(), H5F_SCOPE_LOCAL), "flush " + p, 0);
        bool ok;
        {
          py::gil_scoped_release nogil;
          ok = raw_io(path_, true, off, (char*)arr.data(), nbytes);
        }
        if (!ok) throw H5Err("raw write failed: " + p);
        return;
      }
    }
    if (total) chk(H5Dwrite(d, mt, H5S_ALL, H5S_ALL, H5P_DEFAULT, arr.data()), "write " + p, 0);
  }

  // An empty (uncompressed, contiguous) dataset of `dtype` and `shape`, filled later by
  // write_rows: a writer that receives row blocks one at a time (the sharded prepare's
  // rank-0 writer) never holds the whole matrix.
  void create_dataset(const std::string& p, py::dtype dtype, const std::vector<hsize_t>& dims) {
    if (exists(p)) chk(H5Ldelete(fid(), p.c_str(), H5P_DEFAULT), "unlink " + p, 0);
    if (dtype.kind() == 'b') throw H5Err("create_dataset: bool datasets unsupported");
    const hid_t ft = native_type_for(dtype);
    Hid sp(H5Screate_simple((int)dims.size(), dims.data(), nullptr), H5Sclose);
    Hid dcpl(H5Pcreate(H5P_DATASET_CREATE), H5Pclose);
    H5Pset_fill_time(dcpl, H5D_FILL_TIME_NEVER);
    // allocated at creation: large row blocks then go straight to their file offset
    // (write_rows' raw path)
    H5Pset_layout(dcpl, H5D_CONTIGUOUS);
    H5Pset_alloc_time(dcpl, H5D_ALLOC_TIME_EARLY);
    Hid l = lcpl_intermediate();
    Hid d(chk(H5Dcreate2(fid(), p.c_str(), ft, sp, l, dcpl, H5P_DEFAULT), "create dataset " + p),
          H5Dclose);
  }

  // rows [start, start + value.shape[0]) of an existing dataset (hyperslab along axis 0)
  void write_rows(const std::string& p, long long start, py::array value) {
    py::array arr = py::array::ensure(value, py::array::c_style);
    if (!arr) throw H5Err("write_rows: array must be convertible to C-contiguous");
    Hid d(chk(H5Dopen2(fid(), p.c_str(), H5P_DEFAULT), "open " + p), H5Dclose);
    Hid fsp(H5Dget_space(d), H5Sclose);
    const int nd = H5Sget_simple_extent_ndims(fsp);
    if (nd < 1 || nd != arr.ndim()) throw H5Err("write_rows: rank mismatch for " + p);
    std::vector<hsize_t> dims(nd);
    H5Sget_simple_extent_dims(fsp, dims.data(), nullptr);
    std::vector<hsize_t> cnt = shape_of(arr), off(nd, 0);
    for (int i = 1; i < nd; ++i)
      if (cnt[i] != dims[i]) throw H5Err("write_rows: trailing shape mismatch for " + p);
    if (start < 0 || (hsize_t)start + cnt[0] > dims[0]) throw H5Err("write_rows: rows out of range: " + p);
    if (cnt[0] == 0) return;
    {
      size_t row = (size_t)arr.itemsize();
      for (int i = 1; i < nd; ++i) row *= (size_t)dims[i];
      const size_t nbytes = row * (size_t)cnt[0];
      const hid_t mt = native_type_for(arr.dtype());
      const haddr_t base = nbytes >= kRawMinBytes ? raw_offset(d, mt) : HADDR_UNDEF;
      if (base != HADDR_UNDEF) {
        chk(H5Fflush(fid(), H5F_SCOPE_LOCAL), "flush " + p, 0);
        bool ok;
        {
          py::gil_scoped_release nogil;
          ok = raw_io(path_, true, base + (haddr_t)start * row, (char*)arr.data(), nbytes);
        }
        if (!ok) throw H5Err("raw write failed: " + p);
        return;
      }
    }
    off[0] = (hsize_t)start;
    chk(H5Sselect_hyperslab(fsp, H5S_SELECT_SET, off.data(), nullptr, cnt.data(), nullptr),
        "hyperslab", 0);
    Hid msp(H5Screate_simple(nd, cnt.data(), nullptr), H5Sclose);
    chk(H5Dwrite(d, native_type_for(arr.dtype()), msp, fsp, H5P_DEFAULT, arr.data()),
        "write rows " + p, 0);
  }

  void write_strings(const std::string& p, const std::vector<std::string>& strs) {
    if (exists(p)) chk(H5Ldelete(fid(), p.c_str(), H5P_DEFAULT), "unlink " + p, 0);
    hsize_t n = strs.size();
    std::vector<const char*> ps;
    ps.reserve(n);
    for (auto& s : strs) ps.push_back(s.c_str());
    Hid t = make_vlen_str();
    Hid sp(H5Screate_simple(1, &n, nullptr), H5Sclose);
    Hid l = lcpl_intermediate();
    Hid d(chk(H5Dcreate2(fid(), p.c_str(), t, sp, l, H5P_DEFAULT, H5P_DEFAULT),
              "create str dataset " + p),
          H5Dclose);
    if (n) chk(H5Dwrite(d, t, H5S_ALL, H5S_ALL, H5P_DEFAULT, ps.data()), "write " + p, 0);
  }

  py::tuple shape(const std::string& p) const {
    Hid d(chk(H5Dopen2(fid(), p.c_str(), H5P_DEFAULT), "open " + p), H5Dclose);
    Hid sp(H5Dget_space(d), H5Sclose);
    const int nd = H5Sget_simple_extent_ndims(sp);
    std::vector<hsize_t> dims(nd > 0 ? nd : 0);
    if (nd > 0) H5Sget_simple_extent_dims(sp, dims.data(), nullptr);
    py::tuple t(dims.size());
    for (size_t i = 0; i < dims.size(); ++i) t[i] = py::int_(dims[i]);
    return t;
  }

  std::string dtype_kind(const std::string& p) const {
    Hid d(chk(H5Dopen2(fid(), p.c_str(), H5P_DEFAULT), "open " + p), H5Dclose);
    Hid ft(H5Dget_type(d), H5Tclose);
    const H5T_class_t cls = H5Tget_class(ft);
    if (cls == H5T_STRING) return "string";
    if (is_bool_enum(ft)) return "bool";
    if (cls == H5T_INTEGER || cls == H5T_FLOAT) return "numeric";
    if (cls == H5T_COMPOUND) return "compound";
    return "other";
  }

  // Read a dataset, optionally only rows [start, stop) along axis 0.
  py::object read(const std::string& p, long long start, long long stop) const {
    Hid d(chk(H5Dopen2(fid(), p.c_str(), H5P_DEFAULT), "open " + p), H5Dclose);
    Hid ft(H5Dget_type(d), H5Tclose);
    Hid fsp(H5Dget_space(d), H5Sclose);
    const int nd = H5Sget_simple_extent_ndims(fsp);
    std::vector<hsize_t> dims(nd > 0 ? nd : 0);
    if (nd > 0) H5Sget_simple_extent_dims(fsp, dims.data(), nullptr);
    std::vector<hsize_t> cnt(dims), off(dims.size(), 0);
    const bool sliced = nd >= 1 && (start > 0 || (stop >= 0 && (hsize_t)stop < dims[0]));
    if (sliced) {
      const hsize_t s0 = (hsize_t)std::max<long long>(0, start);
      const hsize_t s1 = stop < 0 ? dims[0] : std::min<hsize_t>(dims[0], (hsize_t)stop);
      off[0] = s0;
      cnt[0] = s1 > s0 ? s1 - s0 : 0;
    }
    hsize_t n = 1;
    for (auto c : cnt) n *= c;
    Hid msp = nd == 0 ? Hid(H5Screate(H5S_SCALAR), H5Sclose)
                      : Hid(H5Screate_simple(nd, cnt.data(), nullptr), H5Sclose);
    if (sliced) {
      chk(H5Sselect_hyperslab(fsp, H5S_SELECT_SET, off.data(), nullptr, cnt.data(), nullptr),
          "hyperslab", 0);
    }
    const hid_t fsel = sliced ? (hid_t)fsp : H5S_ALL;
    const hid_t msel = sliced ? (hid_t)msp : H5S_ALL;
    const H5T_class_t cls = H5Tget_class(ft);
    if (cls == H5T_STRING) {
      if (nd > 1) throw H5Err("multi-dimensional string datasets unsupported: " + p);
      py::list l = read_strings(ft, n, [&](hid_t mt, void* buf) {
        if (n) chk(H5Dread(d, mt, msel, fsel, H5P_DEFAULT, buf), "read " + p, 0);
      });
      if (nd == 0) return l[0];
      return l;
    }
    std::vector<py::ssize_t> shp(cnt.begin(), cnt.end());
    if (is_bool_enum(ft)) {
      py::array_t<bool> out(shp);
      std::vector<int8_t> b(n);
      Hid et = make_bool_enum();
      if (n) chk(H5Dread(d, et, msel, fsel, H5P_DEFAULT, b.data()), "read " + p, 0);
      for (hsize_t i = 0; i < n; ++i) out.mutable_data()[i] = b[i] != 0;
      return out;
    }
    if (cls == H5T_INTEGER || cls == H5T_FLOAT) {
      py::dtype dt = dtype_for_h5(ft);
      py::array out(dt, shp);
      const size_t nbytes = (size_t)n * (size_t)dt.itemsize();
      if (n && nd >= 1 && nbytes >= kRawMinBytes) {
        const haddr_t base = raw_offset(d, mem_type_for(dt));
        if (base != HADDR_UNDEF) {
          size_t row = (size_t)dt.itemsize();
          for (int i = 1; i < nd; ++i) row *= (size_t)dims[i];
          bool ok;
          {
            py::gil_scoped_release nogil;
            ok = raw_io(path_, false, base + (haddr_t)off[0] * row, (char*)out.mutable_data(),
                        nbytes);
          }
          if (ok) return out;            // else: HDF5's own read below
        }
      }
      if (n)
        chk(H5Dread(d, mem_type_for(dt), msel, fsel, H5P_DEFAULT, out.mutable_data()),
            "read " + p, 0);
      if (nd == 0) return out[py::tuple()];
      return out;
    }
    throw H5Err("unsupported dataset type at " + p);
  }

  py::dict attrs(const std::string& p) const {
    Hid o(chk(H5Oopen(fid(), p.c_str(), H5P_DEFAULT), "open " + p), H5Oclose);
    py::dict out;
    const int na = H5Aget_num_attrs(o);
    for (int i = 0; i < na; ++i) {
      Hid a(H5Aopen_by_idx(o, ".", H5_INDEX_NAME, H5_ITER_INC, (hsize_t)i, H5P_DEFAULT,
                           H5P_DEFAULT),
            H5Aclose);
      if (a.id < 0) continue;
      ssize_t len = H5Aget_name(a, 0, nullptr);
      std::string nm(len, '\0');
      H5Aget_name(a, len + 1, &nm[0]);
      out[py::str(nm)] = read_attr_obj(a);
    }
    return out;
  }

  void set_attr(const std::string& p, const std::string& name, py::object value) {
    Hid o(chk(H5Oopen(fid(), p.c_str(), H5P_DEFAULT), "open " + p), H5Oclose);
    write_attr_impl(o, name, value);
  }

 private:
  std::string path_;
  hid_t fid_ = -1;
};

}  // namespace

PYBIND11_MODULE(_h5io, m) {
  m.doc() = "Minimal native HDF5 layer for h5ad I/O (cnmf_torch_amd)";
  py::register_exception<H5Err>(m, "H5Error", PyExc_IOError);
  py::class_<File>(m, "File")
      .def(py::init<const std::string&, const std::string&>(), py::arg("path"),
           py::arg("mode") = "r")
      .def("close", &File::close)
      .def("exists", &File::exists)
      .def("kind", &File::kind)
      .def("list", &File::list)
      .def("create_group", &File::create_group)
      .def("write_array", &File::write_array, py::arg("path"), py::arg("value"),
           py::arg("compression") = 0)
      .def("write_strings", &File::write_strings)
      .def("create_dataset", &File::create_dataset)
      .def("write_rows", &File::write_rows)
      .def("shape", &File::shape)
      .def("dtype_kind", &File::dtype_kind)
      .def("read", &File::read, py::arg("path"), py::arg("start") = 0, py::arg("stop") = -1)
      .def("attrs", &File::attrs)
      .def("set_attr", &File::set_attr)
      .def("__enter__", [](File& f) -> File& { return f; })
      .def("__exit__", [](File& f, py::args) { f.close(); });
  m.attr("HDF5_VERSION") = H5_VERS_INFO;
}
