// Native batch writer of the per-replicate spectra files (cnmf.py:889-892 writes one
// ``spectra.k_%d.iter_%d.df.npz`` per replicate; cNMF factorize produces them by the
// thousand).  Each file is the stored (uncompressed) PKZIP that np.savez writes, with the
// members columns.npy (the gene names, shared by every file), index.npy (1..K) and
// data.npy (K x G float32 spectra).  Files are written atomically (temp file + rename)
// on a pool of native threads, and each one's SHA-256 -- recorded in the replicate
// manifest -- is computed from the bytes in memory, continuing a
// precomputed midstate over the shared prefix.  No Python, no GIL: the Python writer
// spent ~0.1 ms of interpreter time per file under the GIL.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <type_traits>
#include <charconv>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include <unistd.h>
#include <zlib.h>

namespace py = pybind11;

namespace {

// ------------------------------------------------------------------ CRC-32 (zlib polynomial)
struct Crc32 {
  uint32_t t[8][256];
  Crc32() {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = c & 1 ? 0xEDB88320u ^ (c >> 1) : c >> 1;
      t[0][i] = c;
    }
    for (uint32_t i = 0; i < 256; ++i)
      for (int s = 1; s < 8; ++s) t[s][i] = (t[s - 1][i] >> 8) ^ t[0][t[s - 1][i] & 0xFF];
  }
  uint32_t update(uint32_t crc, const uint8_t* p, size_t n) const {
    crc = ~crc;
    while (n >= 8) {  // slicing-by-8
      uint32_t a, b;
      std::memcpy(&a, p, 4);
      std::memcpy(&b, p + 4, 4);
      a ^= crc;
      crc = t[7][a & 0xFF] ^ t[6][(a >> 8) & 0xFF] ^ t[5][(a >> 16) & 0xFF] ^ t[4][a >> 24] ^
            t[3][b & 0xFF] ^ t[2][(b >> 8) & 0xFF] ^ t[1][(b >> 16) & 0xFF] ^ t[0][b >> 24];
      p += 8;
      n -= 8;
    }
    while (n--) crc = t[0][(crc ^ *p++) & 0xFF] ^ (crc >> 8);
    return ~crc;
  }
};
const Crc32& crc_tables() {
  static const Crc32 c;
  return c;
}

// ------------------------------------------------------------------ SHA-256 (FIPS 180-4)
struct Sha256 {
  uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                   0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  uint8_t buf[64];
  size_t blen = 0;
  uint64_t total = 0;

  static uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
  void block(const uint8_t* p) {
    static const uint32_t K[64] = {
        0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4,
        0xab1c5ed5, 0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe,
        0x9bdc06a7, 0xc19bf174, 0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f,
        0x4a7484aa, 0x5cb0a9dc, 0x76f988da, 0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7,
        0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967, 0x27b70a85, 0x2e1b2138, 0x4d2c6dfc,
        0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85, 0xa2bfe8a1, 0xa81a664b,
        0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070, 0x19a4c116,
        0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
        0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7,
        0xc67178f2};
    uint32_t w[64];
    for (int i = 0; i < 16; ++i)
      w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 |
             (uint32_t)p[4 * i + 2] << 8 | p[4 * i + 3];
    for (int i = 16; i < 64; ++i) {
      const uint32_t s0 = rotr(w[i - 15], 7) ^ rotr(w[i - 15], 18) ^ (w[i - 15] >> 3);
      const uint32_t s1 = rotr(w[i - 2], 17) ^ rotr(w[i - 2], 19) ^ (w[i - 2] >> 10);
      w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for (int i = 0; i < 64; ++i) {
      const uint32_t t1 = hh + (rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25)) + ((e & f) ^ (~e & g)) +
                          K[i] + w[i];
      const uint32_t t2 = (rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
      hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
  }
  void update(const uint8_t* p, size_t n) {
    total += n;
    if (blen) {
      const size_t take = std::min(n, 64 - blen);
      std::memcpy(buf + blen, p, take);
      blen += take;
      p += take;
      n -= take;
      if (blen == 64) {
        block(buf);
        blen = 0;
      }
    }
    while (n >= 64) {
      block(p);
      p += 64;
      n -= 64;
    }
    if (n) {
      std::memcpy(buf, p, n);
      blen = n;
    }
  }
  std::string hex() {
    const uint64_t bits = total * 8;
    const uint8_t one = 0x80, zero = 0;
    update(&one, 1);
    while (blen != 56) update(&zero, 1);
    uint8_t len[8];
    for (int i = 0; i < 8; ++i) len[i] = (uint8_t)(bits >> (56 - 8 * i));
    update(len, 8);
    static const char* d = "0123456789abcdef";
    std::string s(64, '0');
    for (int i = 0; i < 8; ++i)
      for (int j = 0; j < 8; ++j) s[i * 8 + j] = d[(h[i] >> (28 - 4 * j)) & 0xF];
    return s;
  }
};

// ------------------------------------------------------------------ stored ZIP records
void put16(std::string& s, uint32_t v) { s.push_back((char)(v & 0xFF)); s.push_back((char)(v >> 8)); }
void put32(std::string& s, uint32_t v) { put16(s, v & 0xFFFF); put16(s, v >> 16); }

std::string local_header(const std::string& name, uint32_t crc, uint32_t size) {
  std::string s;
  put32(s, 0x04034B50); put16(s, 20); put16(s, 0); put16(s, 0); put16(s, 0); put16(s, 33);
  put32(s, crc); put32(s, size); put32(s, size); put16(s, (uint32_t)name.size()); put16(s, 0);
  return s + name;
}
std::string central_record(const std::string& name, uint32_t crc, uint32_t size, uint32_t off) {
  std::string s;
  put32(s, 0x02014B50); put16(s, 20); put16(s, 20); put16(s, 0); put16(s, 0); put16(s, 0);
  put16(s, 33); put32(s, crc); put32(s, size); put32(s, size); put16(s, (uint32_t)name.size());
  put16(s, 0); put16(s, 0); put16(s, 0); put16(s, 0); put32(s, 0600u << 16); put32(s, off);
  return s + name;
}

struct Member {  // a fully encoded member: local header + payload bytes, central record
  std::string local, payload;
  uint32_t crc = 0;
};

}  // namespace

// paths[i] gets members columns (shared) + index (per K) + data (rows offs[i]..offs[i]+ks[i]
// of `data`, with the .npy header data_hdr[K]).  Returns [(sha256 hex, size)].
static std::vector<std::pair<std::string, long long>> write_spectra_batch(
    const std::vector<std::string>& paths, py::array_t<float, py::array::c_style> data,
    const std::vector<long long>& offs, const std::vector<int>& ks, py::bytes columns_npy,
    const std::map<int, py::bytes>& index_npy, const std::map<int, py::bytes>& data_hdr,
    int threads) {
  const size_t n = paths.size();
  if (offs.size() != n || ks.size() != n) throw std::invalid_argument("paths/offs/ks lengths");
  if (data.ndim() != 2) throw std::invalid_argument("data must be 2-D float32");
  const long long rows = data.shape(0), G = data.shape(1);
  for (size_t i = 0; i < n; ++i)
    if (offs[i] < 0 || ks[i] < 1 || offs[i] + ks[i] > rows)
      throw std::invalid_argument("replicate rows out of range");
  const Crc32& crc = crc_tables();
  // shared prefix: the columns member
  Member col;
  col.payload = std::string(columns_npy);
  col.crc = crc.update(0, (const uint8_t*)col.payload.data(), col.payload.size());
  col.local = local_header("columns.npy", col.crc, (uint32_t)col.payload.size());
  Sha256 mid;
  mid.update((const uint8_t*)col.local.data(), col.local.size());
  mid.update((const uint8_t*)col.payload.data(), col.payload.size());
  const uint32_t off_index = (uint32_t)(col.local.size() + col.payload.size());
  std::map<int, Member> idx;
  std::map<int, std::string> hdr;
  for (int K : ks) {
    if (idx.count(K)) continue;
    auto it = index_npy.find(K);
    auto ht = data_hdr.find(K);
    if (it == index_npy.end() || ht == data_hdr.end())
      throw std::invalid_argument("missing index/header bytes for a K");
    Member m;
    m.payload = std::string(it->second);
    m.crc = crc.update(0, (const uint8_t*)m.payload.data(), m.payload.size());
    m.local = local_header("index.npy", m.crc, (uint32_t)m.payload.size());
    idx[K] = std::move(m);
    hdr[K] = std::string(ht->second);
  }
  const float* base = data.data();
  std::vector<std::pair<std::string, long long>> out(n);
  std::vector<std::string> errors(n);
  std::atomic<size_t> next{0};
  auto work = [&]() {
    std::vector<uint8_t> body;
    for (size_t i; (i = next.fetch_add(1)) < n;) {
      const int K = ks[i];
      const Member& im = idx.at(K);
      const std::string& h = hdr.at(K);
      const uint8_t* raw = (const uint8_t*)(base + offs[i] * G);
      const size_t raw_n = (size_t)K * G * sizeof(float);
      uint32_t dcrc = crc.update(0, (const uint8_t*)h.data(), h.size());
      dcrc = crc.update(dcrc, raw, raw_n);
      const uint32_t dsize = (uint32_t)(h.size() + raw_n);
      const uint32_t off_data = off_index + (uint32_t)(im.local.size() + im.payload.size());
      const std::string dlocal = local_header("data.npy", dcrc, dsize);
      const uint32_t off_cd = off_data + (uint32_t)(dlocal.size() + dsize);
      std::string cd = central_record("columns.npy", col.crc, (uint32_t)col.payload.size(), 0) +
                       central_record("index.npy", im.crc, (uint32_t)im.payload.size(), off_index) +
                       central_record("data.npy", dcrc, dsize, off_data);
      std::string end;
      put32(end, 0x06054B50); put16(end, 0); put16(end, 0); put16(end, 3); put16(end, 3);
      put32(end, (uint32_t)cd.size()); put32(end, off_cd); put16(end, 0);
      Sha256 sh = mid;
      auto feed = [&](const void* p, size_t len) { sh.update((const uint8_t*)p, len); };
      feed(im.local.data(), im.local.size());
      feed(im.payload.data(), im.payload.size());
      feed(dlocal.data(), dlocal.size());
      feed(h.data(), h.size());
      feed(raw, raw_n);
      feed(cd.data(), cd.size());
      feed(end.data(), end.size());
      const std::string tmp = paths[i] + ".tmp" + std::to_string(::getpid()) + "_" +
                              std::to_string(i);
      FILE* f = std::fopen(tmp.c_str(), "wb");
      bool ok = f != nullptr;
      auto put = [&](const void* p, size_t len) {
        if (ok && len) ok = std::fwrite(p, 1, len, f) == len;
      };
      put(col.local.data(), col.local.size());
      put(col.payload.data(), col.payload.size());
      put(im.local.data(), im.local.size());
      put(im.payload.data(), im.payload.size());
      put(dlocal.data(), dlocal.size());
      put(h.data(), h.size());
      put(raw, raw_n);
      put(cd.data(), cd.size());
      put(end.data(), end.size());
      if (f && std::fclose(f) != 0) ok = false;
      if (!ok || std::rename(tmp.c_str(), paths[i].c_str()) != 0) {
        std::remove(tmp.c_str());
        errors[i] = "write failed: " + paths[i];
        continue;
      }
      out[i] = {sh.hex(), (long long)off_cd + (long long)cd.size() + (long long)end.size()};
    }
  };
  {
    py::gil_scoped_release nogil;
    const int nt = std::max(1, std::min<int>(threads, (int)n));
    std::vector<std::thread> pool;
    for (int t = 1; t < nt; ++t) pool.emplace_back(work);
    work();
    for (auto& t : pool) t.join();
  }
  for (auto& e : errors)
    if (!e.empty()) throw std::runtime_error(e);
  return out;
}

// ------------------------------------------------------------------ batch reader
// Inverse of write_spectra_batch for `combine` (cnmf.py:895-920 reads every replicate
// file of a K back): each stored npz is parsed natively -- end-of-central-directory,
// central records, local headers, the data.npy header (<f4, C order, (K, G)) -- on a pool
// of threads, and the spectra are copied into ONE float32 matrix.  The columns.npy
// payloads must be byte-identical to the first file's.  Anything else (a deflated member,
// another dtype, object arrays from the original cnmf, different gene-name bytes) is
// reported as unsupported, and the caller takes the numpy path for the batch.
namespace {

uint32_t get16(const uint8_t* p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8); }
uint32_t get32(const uint8_t* p) { return get16(p) | (get16(p + 2) << 16); }

struct NpzFile {
  std::vector<uint8_t> bytes;
  const uint8_t* data = nullptr;   // data.npy payload (float32, K x G)
  const uint8_t* cols = nullptr;   // columns.npy payload
  size_t cols_n = 0;
  long long K = 0, G = 0;
  std::string err;                 // non-empty: unsupported / unreadable
};

bool read_all(const std::string& path, std::vector<uint8_t>& out) {
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) return false;
  std::fseek(f, 0, SEEK_END);
  const long n = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  bool ok = n > 0;
  if (ok) {
    out.resize((size_t)n);
    ok = std::fread(out.data(), 1, (size_t)n, f) == (size_t)n;
  }
  std::fclose(f);
  return ok;
}

// shape (K, G) of a float32 C-order .npy payload; false if it is anything else
bool npy_f4_2d(const uint8_t* p, size_t n, long long& K, long long& G, size_t& hdr) {
  if (n < 10 || std::memcmp(p, "\x93NUMPY", 6) != 0) return false;
  const int major = p[6];
  size_t hl, start;
  if (major == 1) { hl = get16(p + 8); start = 10; }
  else if (major == 2 || major == 3) { if (n < 12) return false; hl = get32(p + 8); start = 12; }
  else return false;
  if (start + hl > n) return false;
  const std::string h((const char*)p + start, hl);
  if (h.find("'descr': '<f4'") == std::string::npos) return false;
  if (h.find("'fortran_order': False") == std::string::npos) return false;
  const size_t sp = h.find("'shape': (");
  if (sp == std::string::npos) return false;
  long long a = -1, b = -1;
  if (std::sscanf(h.c_str() + sp + 10, "%lld, %lld)", &a, &b) != 2 || a < 1 || b < 1) return false;
  hdr = start + hl;
  // a * b * 4 must not wrap: reject shapes beyond the payload before multiplying
  if ((unsigned long long)a > (n / 4) || (unsigned long long)b > (n / 4) / (size_t)a) return false;
  if (hdr + (size_t)a * (size_t)b * 4 > n) return false;
  K = a;
  G = b;
  return true;
}

void parse_npz(const std::string& path, NpzFile& f) {
  if (!read_all(path, f.bytes)) { f.err = "unreadable: " + path; return; }
  const uint8_t* b = f.bytes.data();
  const size_t n = f.bytes.size();
  if (n < 22) { f.err = "not a zip: " + path; return; }
  size_t eocd = std::string::npos;
  for (size_t i = n - 22 + 1; i-- > (n > 65557 ? n - 65557 : 0);)
    if (get32(b + i) == 0x06054B50) { eocd = i; break; }
  if (eocd == std::string::npos) { f.err = "no end of central directory: " + path; return; }
  const uint32_t entries = get16(b + eocd + 10);
  size_t cd = get32(b + eocd + 16);
  // every offset below is size_t arithmetic on values read from the file, checked
  // against the buffer before it is dereferenced (a truncated or malformed file is
  // reported as unsupported and handed to the numpy path, never read out of bounds)
  for (uint32_t e = 0; e < entries; ++e) {
    if (cd > n || n - cd < 46 || get32(b + cd) != 0x02014B50) {
      f.err = "bad central record: " + path;
      return;
    }
    const size_t method = get16(b + cd + 10), csize = get32(b + cd + 20);
    const size_t nl = get16(b + cd + 28), xl = get16(b + cd + 30), cl = get16(b + cd + 32);
    const size_t lo = get32(b + cd + 42);
    if (n - cd - 46 < nl + xl + cl) { f.err = "bad central record: " + path; return; }
    const std::string name((const char*)b + cd + 46, nl);
    cd += 46 + nl + xl + cl;
    if (name != "data.npy" && name != "columns.npy") continue;
    if (method != 0) { f.err = "compressed member: " + path; return; }
    if (lo > n || n - lo < 30 || get32(b + lo) != 0x04034B50) {
      f.err = "bad local header: " + path;
      return;
    }
    const size_t pay = lo + 30 + (size_t)get16(b + lo + 26) + (size_t)get16(b + lo + 28);
    if (pay > n || n - pay < csize) { f.err = "truncated member: " + path; return; }
    if (name == "columns.npy") {
      f.cols = b + pay;
      f.cols_n = csize;
    } else {
      size_t hdr = 0;
      if (!npy_f4_2d(b + pay, csize, f.K, f.G, hdr)) { f.err = "data is not float32 2-D: " + path; return; }
      f.data = b + pay + hdr;
    }
  }
  if (!f.data || !f.cols) f.err = "missing data/columns member: " + path;
}

}  // namespace

// -> (data (sum K, G) float32, [K per file], columns.npy bytes of the first file); raises
// ValueError("unsupported: ...") when a file needs the numpy path
static py::tuple read_spectra_batch(const std::vector<std::string>& paths, int threads) {
  const size_t n = paths.size();
  if (n == 0) throw std::invalid_argument("no files");
  std::vector<NpzFile> files(n);
  std::atomic<size_t> next{0};
  auto run = [&](auto&& fn) {
    next = 0;
    py::gil_scoped_release nogil;
    const int nt = std::max(1, std::min<int>(threads, (int)n));
    std::vector<std::thread> pool;
    for (int t = 1; t < nt; ++t) pool.emplace_back(fn);
    fn();
    for (auto& t : pool) t.join();
  };
  run([&]() {
    for (size_t i; (i = next.fetch_add(1)) < n;) parse_npz(paths[i], files[i]);
  });
  long long rows = 0;
  std::vector<long long> offs(n);
  std::vector<int> ks(n);
  for (size_t i = 0; i < n; ++i) {
    const NpzFile& f = files[i];
    if (!f.err.empty()) throw py::value_error("unsupported: " + f.err);
    if (f.G != files[0].G || f.cols_n != files[0].cols_n ||
        std::memcmp(f.cols, files[0].cols, f.cols_n) != 0)
      throw py::value_error("unsupported: gene columns differ from the first file: " + paths[i]);
    offs[i] = rows;
    ks[i] = (int)f.K;
    rows += f.K;
  }
  const long long G = files[0].G;
  py::array_t<float> out({rows, G});
  float* dst = out.mutable_data();
  run([&]() {
    for (size_t i; (i = next.fetch_add(1)) < n;)
      std::memcpy(dst + offs[i] * G, files[i].data, (size_t)files[i].K * G * sizeof(float));
  });
  py::bytes cols((const char*)files[0].cols, files[0].cols_n);
  return py::make_tuple(out, ks, cols);
}

static std::string sha256_hex(py::bytes b) {
  std::string s(b);
  Sha256 h;
  h.update((const uint8_t*)s.data(), s.size());
  return h.hex();
}

static unsigned crc32_bytes(py::bytes b) {
  std::string s(b);
  return crc_tables().update(0, (const uint8_t*)s.data(), s.size());
}

// ------------------------------------------------------------------------ TSV writer
// DataFrame.to_csv(sep="\t") of an all-float frame (cnmf.py:35-36 save_df_to_text), byte
// for byte: every value in its shortest round-trip form -- Python's repr for float64
// (scientific below a decimal exponent of -4 or from 16 on), numpy's str for float32
// (scientific below 1e-4 or from 1e16 in magnitude) -- NaN as the empty string, integral
// values with ".0".  Rows are formatted on native threads.
namespace {

void fmt_value(double v, bool f32, std::string& out) {
  if (std::isnan(v)) return;
  if (std::isinf(v)) {
    out += v > 0 ? "inf" : "-inf";
    return;
  }
  char buf[64];
  std::to_chars_result r = f32 ? std::to_chars(buf, buf + 64, (float)v, std::chars_format::scientific)
                               : std::to_chars(buf, buf + 64, v, std::chars_format::scientific);
  const char* p = buf;
  const char* end = r.ptr;
  std::string neg;
  if (*p == '-') {
    neg = "-";
    ++p;
  }
  std::string dig;
  while (p < end && *p != 'e') {
    if (*p != '.') dig += *p;
    ++p;
  }
  int ex = 0;                                // "e-05" / "e+16": parse within [p, end)
  if (p < end) {
    const char* q = p + 1;
    const bool eneg = q < end && *q == '-';
    if (q < end && (*q == '-' || *q == '+')) ++q;
    std::from_chars(q, end, ex);
    if (eneg) ex = -ex;
  }
  const double a = std::fabs(v);
  const bool sci = (a != 0.0) && (f32 ? (a < 1e-4 || a >= 1e16) : (ex < -4 || ex >= 16));
  out += neg;
  if (sci) {
    out += dig[0];
    if (dig.size() > 1) {
      out += '.';
      out.append(dig, 1, std::string::npos);
    }
    char eb[16];
    std::snprintf(eb, sizeof eb, "e%c%02d", ex < 0 ? '-' : '+', ex < 0 ? -ex : ex);
    out += eb;
  } else if (ex >= 0) {
    if ((int)dig.size() <= ex + 1) {
      out += dig;
      out.append(ex + 1 - dig.size(), '0');
      out += ".0";
    } else {
      out.append(dig, 0, ex + 1);
      out += '.';
      out.append(dig, ex + 1, std::string::npos);
    }
  } else {
    out += "0.";
    out.append(-ex - 1, '0');
    out += dig;
  }
}

}  // namespace

static void write_tsv(const std::string& path, const std::string& corner,
                      const std::vector<std::string>& columns,
                      const std::vector<std::string>& index, py::array data, int threads) {
  const bool f32 = py::isinstance<py::array_t<float>>(data);
  if (!f32 && !py::isinstance<py::array_t<double>>(data))
    throw std::invalid_argument("write_tsv: float32 or float64 data");
  if (data.ndim() != 2) throw std::invalid_argument("write_tsv: 2-D data");
  const size_t n = data.shape(0), g = data.shape(1);
  if (n != index.size() || g != columns.size())
    throw std::invalid_argument("write_tsv: shape does not match index / columns");
  py::array c = py::array::ensure(data, py::array::c_style);
  const char* base = (const char*)c.data();
  std::vector<std::string> rows(n);
  std::atomic<size_t> next{0};
  {
    py::gil_scoped_release nogil;
    auto work = [&]() {
      for (size_t i; (i = next.fetch_add(64)) < n;) {
        for (size_t r = i; r < std::min(n, i + 64); ++r) {
          std::string& s = rows[r];
          s.reserve(g * 12 + index[r].size() + 2);
          s += index[r];
          for (size_t j = 0; j < g; ++j) {
            s += '\t';
            const double v = f32 ? (double)((const float*)base)[r * g + j]
                                 : ((const double*)base)[r * g + j];
            fmt_value(v, f32, s);
          }
          s += '\n';
        }
      }
    };
    const int nt = std::max(1, std::min<int>(threads, (int)(n / 64) + 1));
    std::vector<std::thread> pool;
    for (int t = 1; t < nt; ++t) pool.emplace_back(work);
    work();
    for (auto& t : pool) t.join();
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) throw std::runtime_error("write_tsv: cannot open " + path);
    std::string head = corner;
    for (const auto& col : columns) {
      head += '\t';
      head += col;
    }
    head += '\n';
    bool ok = std::fwrite(head.data(), 1, head.size(), f) == head.size();
    for (const auto& s : rows) ok = ok && std::fwrite(s.data(), 1, s.size(), f) == s.size();
    ok = (std::fclose(f) == 0) && ok;
    if (!ok) throw std::runtime_error("write_tsv: write failed: " + path);
  }
}

// ------------------------------------------------------------------------ CSR statistics
// Column mean and ddof=0 variance of a CSR matrix by sklearn's corrected two-pass
// algorithm (sklearn/utils/sparsefuncs_fast.pyx _csr_mean_variance_axis0, unit weights;
// cnmf.py:128-131 runs it through StandardScaler): the same float64 operations in the
// same order (row-major over the stored entries), hence the same bits -- at C++ speed and
// without sklearn's ~1 s import on the prepare path.
template <typename T, typename I>
static void csr_mean_var_impl(const T* data, const I* indices, long long nnz, long long n_rows,
                              long long G, double* mean, double* var) {
  std::vector<double> corr(G, 0.0);
  std::vector<long long> cnt(G, 0);
  for (long long j = 0; j < G; ++j) mean[j] = var[j] = 0.0;
  for (long long e = 0; e < nnz; ++e) {
    const I c = indices[e];
    mean[c] += (double)data[e];
    cnt[c] += 1;
  }
  const double n = (double)n_rows;
  for (long long j = 0; j < G; ++j) mean[j] /= n;
  for (long long e = 0; e < nnz; ++e) {
    const I c = indices[e];
    const double d = (double)data[e] - mean[c];
    corr[c] += d;
    var[c] += d * d;
  }
  for (long long j = 0; j < G; ++j) {
    const bool miss = cnt[j] != n_rows;
    if (miss) corr[j] -= (n - (double)cnt[j]) * mean[j];
    corr[j] = corr[j] * corr[j] / n;
    if (miss) var[j] += (n - (double)cnt[j]) * (mean[j] * mean[j]);   // sklearn: means**2
    var[j] = (var[j] - corr[j]) / n;
  }
}

static py::tuple csr_mean_var(py::array data, py::array indices, long long n_rows, long long G) {
  py::array_t<double> mean(G), var(G);
  const long long nnz = data.size();
  if (indices.size() != nnz) throw std::invalid_argument("csr_mean_var: data / indices sizes");
  py::array d = py::array::ensure(data, py::array::c_style);
  py::array ix = py::array::ensure(indices, py::array::c_style);
  double* m = mean.mutable_data();
  double* v = var.mutable_data();
  const bool i64 = py::isinstance<py::array_t<long long>>(ix) || py::isinstance<py::array_t<int64_t>>(ix);
  if (!i64 && !py::isinstance<py::array_t<int>>(ix))
    throw std::invalid_argument("csr_mean_var: int32 or int64 indices");
  auto run = [&](auto tag) {
    using T = decltype(tag);
    const T* dp = (const T*)d.data();
    py::gil_scoped_release nogil;
    if (i64) csr_mean_var_impl(dp, (const long long*)ix.data(), nnz, n_rows, G, m, v);
    else csr_mean_var_impl(dp, (const int*)ix.data(), nnz, n_rows, G, m, v);
  };
  if (py::isinstance<py::array_t<double>>(d)) run(double{});
  else if (py::isinstance<py::array_t<float>>(d)) run(float{});
  else throw std::invalid_argument("csr_mean_var: float32 or float64 data");
  return py::make_tuple(mean, var);
}

// data[e] *= scale[row(e)] in the data's own precision (normalize_total's row scaling:
// float32 data times the float32-rounded factor, as numpy does), rows on native threads
static void csr_scale_rows(py::array data, py::array indptr, py::array_t<double> scale,
                           int threads) {
  py::array ip = py::array::ensure(indptr, py::array::c_style);
  const long long n = scale.size();
  if (ip.size() != n + 1) throw std::invalid_argument("csr_scale_rows: indptr / scale sizes");
  std::vector<long long> ptr(n + 1);
  if (py::isinstance<py::array_t<int>>(ip)) {
    const int* q = (const int*)ip.data();
    for (long long i = 0; i <= n; ++i) ptr[i] = q[i];
  } else {
    const long long* q = (const long long*)ip.data();
    for (long long i = 0; i <= n; ++i) ptr[i] = q[i];
  }
  const double* sc = scale.data();
  auto go = [&](auto* dp) {
    using T = std::remove_pointer_t<decltype(dp)>;
    std::atomic<long long> next{0};
    py::gil_scoped_release nogil;
    auto work = [&]() {
      for (long long r0; (r0 = next.fetch_add(256)) < n;)
        for (long long r = r0; r < std::min(n, r0 + 256); ++r) {
          const T f = (T)sc[r];
          for (long long e = ptr[r]; e < ptr[r + 1]; ++e) dp[e] = dp[e] * f;
        }
    };
    const int nt = std::max(1, std::min<int>(threads, (int)(n / 256) + 1));
    std::vector<std::thread> pool;
    for (int t = 1; t < nt; ++t) pool.emplace_back(work);
    work();
    for (auto& t : pool) t.join();
  };
  if (!(data.flags() & py::array::c_style)) throw std::invalid_argument("csr_scale_rows: contiguous data");
  if (py::isinstance<py::array_t<float>>(data)) go((float*)data.mutable_data());
  else if (py::isinstance<py::array_t<double>>(data)) go((double*)data.mutable_data());
  else throw std::invalid_argument("csr_scale_rows: float32 or float64 data");
}

// PNG (RGBA8, filter 0 on every row) of an (H, W, 4) uint8 image: the deflate stream is
// compressed in row bands on `threads` threads, each band a raw deflate ending in a full
// flush (the last in Z_FINISH), so the concatenated bands form one valid stream (the pigz
// construction); the zlib adler32 over the whole filtered image closes it.  Chunks as
// matplotlib's Agg/PIL output: IHDR, pHYs, tEXt "Software", IDAT, IEND.
static void png_chunk(std::string& out, const char* tag, const std::string& data) {
  const uint32_t n = (uint32_t)data.size();
  const unsigned char len[4] = {(unsigned char)(n >> 24), (unsigned char)(n >> 16),
                                (unsigned char)(n >> 8), (unsigned char)n};
  out.append((const char*)len, 4);
  out.append(tag, 4);
  out += data;
  uLong c = crc32(0L, (const Bytef*)tag, 4);
  c = crc32(c, (const Bytef*)data.data(), (uInt)data.size());
  const unsigned char cb[4] = {(unsigned char)(c >> 24), (unsigned char)(c >> 16),
                               (unsigned char)(c >> 8), (unsigned char)c};
  out.append((const char*)cb, 4);
}

static std::string be32(uint32_t v) {
  const char b[4] = {(char)(v >> 24), (char)(v >> 16), (char)(v >> 8), (char)v};
  return std::string(b, 4);
}

static void write_png_rgba(const std::string& path, py::array_t<uint8_t, py::array::c_style> img,
                           double dpi, const std::string& software, int level, int threads) {
  if (img.ndim() != 3 || img.shape(2) != 4) throw std::invalid_argument("write_png_rgba: (H, W, 4)");
  const long long h = img.shape(0), w = img.shape(1), row = 1 + 4 * w;
  const uint8_t* src = img.data();
  std::string out;
  {
    py::gil_scoped_release nogil;
    std::vector<uint8_t> raw((size_t)(h * row));
    for (long long r = 0; r < h; ++r) {
      raw[(size_t)(r * row)] = 0;
      std::memcpy(&raw[(size_t)(r * row + 1)], src + r * 4 * w, (size_t)(4 * w));
    }
    const int nt = std::max(1, std::min<int>(threads, (int)std::max<long long>(1, h / 16)));
    const long long band = (h + nt - 1) / nt;
    std::vector<std::string> parts(nt);
    std::vector<uLong> adl(nt, 1);
    std::vector<int> err(nt, 0);
    auto work = [&](int t) {
      const long long r0 = t * band, r1 = std::min(h, r0 + band);
      if (r0 >= r1) return;
      const Bytef* in = raw.data() + r0 * row;
      const uInt n = (uInt)((r1 - r0) * row);
      adl[t] = adler32(1L, in, n);
      z_stream zs;
      std::memset(&zs, 0, sizeof(zs));
      if (deflateInit2(&zs, level, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK) { err[t] = 1; return; }
      std::string& o = parts[t];
      o.resize(deflateBound(&zs, n) + 64);
      zs.next_in = const_cast<Bytef*>(in);
      zs.avail_in = n;
      zs.next_out = (Bytef*)&o[0];
      zs.avail_out = (uInt)o.size();
      const int rc = deflate(&zs, r1 == h ? Z_FINISH : Z_FULL_FLUSH);
      if ((r1 == h && rc != Z_STREAM_END) || (r1 != h && rc != Z_OK) || zs.avail_in != 0) err[t] = 1;
      o.resize(o.size() - zs.avail_out);
      deflateEnd(&zs);
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < nt; ++t) pool.emplace_back(work, t);
    work(0);
    for (auto& t : pool) t.join();
    for (int t = 0; t < nt; ++t)
      if (err[t]) throw std::runtime_error("write_png_rgba: deflate failed");
    uLong ad = adl[0];
    for (int t = 1; t < nt; ++t) {
      const long long r0 = t * band, r1 = std::min(h, r0 + band);
      if (r0 < r1) ad = adler32_combine(ad, adl[t], (z_off_t)((r1 - r0) * row));
    }
    std::string idat("\x78\x01", 2);
    for (auto& pt : parts) idat += pt;
    idat += be32((uint32_t)ad);
    const uint32_t ppm = (uint32_t)std::llround(dpi / 0.0254);
    out.append("\x89PNG\r\n\x1a\n", 8);
    std::string ihdr = be32((uint32_t)w) + be32((uint32_t)h);
    ihdr += std::string("\x08\x06\x00\x00\x00", 5);
    png_chunk(out, "IHDR", ihdr);
    png_chunk(out, "pHYs", be32(ppm) + be32(ppm) + std::string("\x01", 1));
    png_chunk(out, "tEXt", std::string("Software") + std::string("\0", 1) + software);
    png_chunk(out, "IDAT", idat);
    png_chunk(out, "IEND", std::string());
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) throw std::runtime_error("write_png_rgba: cannot open " + path);
    const size_t wr = std::fwrite(out.data(), 1, out.size(), f);
    const int cl = std::fclose(f);
    if (wr != out.size() || cl != 0) throw std::runtime_error("write_png_rgba: write failed " + path);
  }
}

// ---------------------------------------------------------------------------------------
// Exact column moments (sum x, sum x^2 per column) as integer digit vectors: every value
// x = +-m 2^e (m < 2^53) is added EXACTLY into base-2^32 digits held in int64 (each add
// contributes < 2^32 per digit, so 2^31 adds per digit cannot overflow).  Integer sums
// are associative: any row partition -- threads, row blocks, the ranks of a sharded
// prepare all-reducing the digits -- gives the identical totals, from which mean and
// variance are rounded ONCE (cnmf_torch_amd.models.hvg.exact_mean_var).  Window: |x| in
// [2^-126, 2^127] (float32's normal range); anything else is counted in `outside` and the
// caller falls back to floating-point statistics.
constexpr int kExLsb1 = -192, kExD1 = 13;     // sums: bits [2^-192, 2^224)
constexpr int kExLsb2 = -384, kExD2 = 25;     // squares: bits [2^-384, 2^416)

static inline bool ex_add(double x, long long* d1, long long* d2) {
  if (x == 0.0) return true;
  const double ax = std::fabs(x);
  if (!(ax >= 0x1p-126 && ax <= 0x1p127)) return false;
  int E;
  const double f = std::frexp(ax, &E);                  // ax = f 2^E, f in [0.5, 1)
  const uint64_t m = (uint64_t)std::ldexp(f, 53);        // exact: 53-bit integer
  const int e = E - 53;                                  // ax = m 2^e
  const long long sg = x < 0.0 ? -1 : 1;
  {
    const int s = e - kExLsb1, dd = s >> 5, o = s & 31;
    const unsigned __int128 v = (unsigned __int128)m << o;
    d1[dd] += sg * (long long)(uint64_t)(v & 0xFFFFFFFFu);
    d1[dd + 1] += sg * (long long)(uint64_t)((v >> 32) & 0xFFFFFFFFu);
    d1[dd + 2] += sg * (long long)(uint64_t)(v >> 64);
  }
  {
    const unsigned __int128 mm = (unsigned __int128)m * m;   // < 2^106
    const int s = 2 * e - kExLsb2, dd = s >> 5, o = s & 31;
    const unsigned __int128 lo = mm << o;                      // low 128 bits
    const uint64_t hi = o ? (uint64_t)(mm >> (128 - o)) : 0;   // bits >= 128
    d2[dd] += (long long)(uint64_t)(lo & 0xFFFFFFFFu);
    d2[dd + 1] += (long long)(uint64_t)((lo >> 32) & 0xFFFFFFFFu);
    d2[dd + 2] += (long long)(uint64_t)((lo >> 64) & 0xFFFFFFFFu);
    d2[dd + 3] += (long long)(uint64_t)(lo >> 96);
    d2[dd + 4] += (long long)hi;
  }
  return true;
}

// CSR (any row partition): entries [0, nnz) with column indices; threads split the entries
// and each keeps private digits, summed at the end (integer: exact in any order)
template <typename T, typename I>
static long long ex_csr_impl(const T* data, const I* idx, long long nnz, long long G,
                             long long* out1, long long* out2, int threads) {
  threads = std::max(1, std::min(threads, (int)std::max(1LL, nnz / 65536)));
  std::vector<std::vector<long long>> p1(threads), p2(threads);
  std::vector<long long> bad(threads, 0);
  std::vector<std::thread> pool;
  for (int t = 0; t < threads; ++t) {
    pool.emplace_back([&, t] {
      p1[t].assign(G * kExD1, 0);
      p2[t].assign(G * kExD2, 0);
      const long long a = nnz * t / threads, b = nnz * (t + 1) / threads;
      for (long long e = a; e < b; ++e) {
        const long long c = (long long)idx[e];
        if (!ex_add((double)data[e], p1[t].data() + c * kExD1, p2[t].data() + c * kExD2))
          ++bad[t];
      }
    });
  }
  for (auto& th : pool) th.join();
  long long nb = 0;
  for (int t = 0; t < threads; ++t) {
    nb += bad[t];
    for (long long i = 0; i < G * kExD1; ++i) out1[i] += p1[t][i];
    for (long long i = 0; i < G * kExD2; ++i) out2[i] += p2[t][i];
  }
  return nb;
}

// dense row-major (rows x G, row stride ld): rows split over threads
template <typename T>
static long long ex_dense_impl(const T* X, long long rows, long long G, long long ld,
                               long long* out1, long long* out2, int threads) {
  threads = std::max(1, std::min(threads, (int)std::max(1LL, rows * G / 65536)));
  std::vector<std::vector<long long>> p1(threads), p2(threads);
  std::vector<long long> bad(threads, 0);
  std::vector<std::thread> pool;
  for (int t = 0; t < threads; ++t) {
    pool.emplace_back([&, t] {
      p1[t].assign(G * kExD1, 0);
      p2[t].assign(G * kExD2, 0);
      const long long a = rows * t / threads, b = rows * (t + 1) / threads;
      for (long long r = a; r < b; ++r)
        for (long long c = 0; c < G; ++c)
          if (!ex_add((double)X[r * ld + c], p1[t].data() + c * kExD1, p2[t].data() + c * kExD2))
            ++bad[t];
    });
  }
  for (auto& th : pool) th.join();
  long long nb = 0;
  for (int t = 0; t < threads; ++t) {
    nb += bad[t];
    for (long long i = 0; i < G * kExD1; ++i) out1[i] += p1[t][i];
    for (long long i = 0; i < G * kExD2; ++i) out2[i] += p2[t][i];
  }
  return nb;
}

// returns (digits1 int64 (G, D1), digits2 int64 (G, D2), values outside the window)
static py::tuple exact_col_moments(py::array data, py::object indices, long long G, int threads) {
  py::array_t<long long> d1({G, (long long)kExD1}), d2({G, (long long)kExD2});
  std::memset(d1.mutable_data(), 0, sizeof(long long) * G * kExD1);
  std::memset(d2.mutable_data(), 0, sizeof(long long) * G * kExD2);
  py::array d = py::array::ensure(data, py::array::c_style);
  long long bad = 0;
  auto run_dense = [&](auto tag) {
    using T = decltype(tag);
    if (d.ndim() != 2 || d.shape(1) != G) throw std::invalid_argument("exact_col_moments: (rows, G)");
    const T* xp = (const T*)d.data();
    const long long rows = d.shape(0);
    py::gil_scoped_release nogil;
    bad = ex_dense_impl(xp, rows, G, G, d1.mutable_data(), d2.mutable_data(), threads);
  };
  if (indices.is_none()) {
    if (py::isinstance<py::array_t<double>>(d)) run_dense(double{});
    else if (py::isinstance<py::array_t<float>>(d)) run_dense(float{});
    else throw std::invalid_argument("exact_col_moments: float32 or float64 data");
    return py::make_tuple(d1, d2, bad);
  }
  py::array ix = py::array::ensure(indices, py::array::c_style);
  const long long nnz = d.size();
  if (ix.size() != nnz) throw std::invalid_argument("exact_col_moments: data / indices sizes");
  const bool i64 = py::isinstance<py::array_t<long long>>(ix) || py::isinstance<py::array_t<int64_t>>(ix);
  if (!i64 && !py::isinstance<py::array_t<int>>(ix))
    throw std::invalid_argument("exact_col_moments: int32 or int64 indices");
  auto run = [&](auto tag) {
    using T = decltype(tag);
    const T* dp = (const T*)d.data();
    py::gil_scoped_release nogil;
    if (i64) bad = ex_csr_impl(dp, (const long long*)ix.data(), nnz, G, d1.mutable_data(), d2.mutable_data(), threads);
    else bad = ex_csr_impl(dp, (const int*)ix.data(), nnz, G, d1.mutable_data(), d2.mutable_data(), threads);
  };
  if (py::isinstance<py::array_t<double>>(d)) run(double{});
  else if (py::isinstance<py::array_t<float>>(d)) run(float{});
  else throw std::invalid_argument("exact_col_moments: float32 or float64 data");
  return py::make_tuple(d1, d2, bad);
}

PYBIND11_MODULE(_npzio, m) {
  m.doc() = "cnmf_torch_amd native replicate-file writer/reader (stored npz, crc32, sha256)";
  m.def("write_spectra_batch", &write_spectra_batch, py::arg("paths"), py::arg("data"),
        py::arg("offs"), py::arg("ks"), py::arg("columns_npy"), py::arg("index_npy"),
        py::arg("data_hdr"), py::arg("threads") = 16);
  m.def("read_spectra_batch", &read_spectra_batch, py::arg("paths"), py::arg("threads") = 16);
  m.def("write_tsv", &write_tsv, py::arg("path"), py::arg("corner"), py::arg("columns"),
        py::arg("index"), py::arg("data"), py::arg("threads") = 16);
  m.def("csr_mean_var", &csr_mean_var);
  m.def("exact_col_moments", &exact_col_moments, py::arg("data"), py::arg("indices"),
        py::arg("G"), py::arg("threads") = 16);
  m.attr("EXACT_LSB1") = kExLsb1;
  m.attr("EXACT_LSB2") = kExLsb2;
  m.def("csr_scale_rows", &csr_scale_rows, py::arg("data"), py::arg("indptr"), py::arg("scale"),
        py::arg("threads") = 16);
  m.def("sha256_hex", &sha256_hex);
  m.def("crc32", &crc32_bytes);
  m.def("write_png_rgba", &write_png_rgba, py::arg("path"), py::arg("img"), py::arg("dpi"),
        py::arg("software"), py::arg("level") = 1, py::arg("threads") = 8);
}
