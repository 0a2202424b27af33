// parquet_gzip.cpp -- adamSave's GZIP part files (SURVEY.md §8 f2;
// adam-core/.../rdd/AdamRDDFunctions.scala:37-48 writes ADAMRecords through
// parquet-mr with the codec of ParquetArgs, adam-cli/.../cli/ParquetArgs.scala:27:
// CompressionCodecName.GZIP by default).
//
// A part file arrives as a Parquet file written UNCOMPRESSED in memory by
// Arrow's writer (schema, encodings, dictionary pages, statistics: everything
// but the codec), and is written out with every page gzip-compressed -- the
// page headers, column-chunk metadata and footer re-encoded with the new
// sizes and offsets.  Reading back gives the same table as Arrow's own GZIP
// writer.
//
// Compression per column:
//  * the per-base strings (qual, sequence): one dynamic-Huffman DEFLATE block
//    per page, no string matching.  Their bytes are quality and base letters
//    whose redundancy is their skewed letter frequencies, which the Huffman
//    code takes; zlib's level 6 spends most of its time searching matches
//    that barely pay (measured on synthetic 100-bp reads, bytes out / in:
//    qual 0.539 zlib-6, 0.502 here; sequence 0.294 / 0.28 -- zlib's own
//    Z_HUFFMAN_ONLY gives the same sizes), at memory speed;
//  * every other column: libdeflate (loaded at run time; zlib when absent) at
//    the given level -- zlib's default 6, as Hadoop's GzipCodec.
// A gzip member per page (RFC 1952), as parquet-mr's GzipCodec writes.
//
// The Thrift compact protocol (parquet.thrift's FileMetaData / PageHeader) is
// handled generically: structures are parsed into trees and written back
// field by field, so fields this code does not know survive unchanged.

namespace pqgz {

// ---------------------------------------------------------------- thrift ----
enum : uint8_t {
  kTStop = 0, kTTrue = 1, kTFalse = 2, kTByte = 3, kTI16 = 4, kTI32 = 5, kTI64 = 6, kTDouble = 7,
  kTBinary = 8, kTList = 9, kTSet = 10, kTMap = 11, kTStruct = 12
};

struct TVal;
struct TField;
struct TVal {
  uint8_t type = kTStop;         // kT*: kTTrue / kTFalse for booleans
  int64_t i = 0;                 // integers, booleans (0/1)
  double d = 0;
  std::string bin;
  uint8_t etype = 0;             // list / set element type; map key type
  uint8_t vtype = 0;             // map value type
  std::vector<TVal> elems;       // list / set elements; map: key, value, key, value ...
  std::vector<TField> fields;    // struct
};
struct TField {
  int16_t id;
  TVal v;
};

struct Reader {
  const uint8_t* p;
  const uint8_t* end;
  bool ok = true;
  uint8_t byte() {
    if (p >= end) {
      ok = false;
      return 0;
    }
    return *p++;
  }
  uint64_t varint() {
    uint64_t v = 0;
    for (int s = 0; s < 64; s += 7) {
      const uint8_t b = byte();
      v |= (uint64_t)(b & 0x7F) << s;
      if (!(b & 0x80)) return v;
    }
    ok = false;
    return 0;
  }
  int64_t zigzag() {
    const uint64_t v = varint();
    return (int64_t)(v >> 1) ^ -(int64_t)(v & 1);
  }
  void value(uint8_t type, TVal& v, int depth);
  void fields(std::vector<TField>& out, int depth) {
    int16_t last = 0;
    while (ok) {
      const uint8_t h = byte();
      if (!ok) return;
      const uint8_t type = h & 0x0F;
      if (type == kTStop) return;
      const int delta = h >> 4;
      const int16_t id = delta ? (int16_t)(last + delta) : (int16_t)zigzag();
      TField f{id, {}};
      value(type, f.v, depth + 1);
      out.push_back(std::move(f));
      last = id;
    }
  }
};

void Reader::value(uint8_t type, TVal& v, int depth) {
  if (depth > 64) {
    ok = false;
    return;
  }
  v.type = type;
  switch (type) {
    case kTTrue: v.i = 1; break;
    case kTFalse: v.i = 0; break;
    case kTByte: v.i = (int8_t)byte(); break;
    case kTI16:
    case kTI32:
    case kTI64: v.i = zigzag(); break;
    case kTDouble:
      if (end - p < 8) {
        ok = false;
        return;
      }
      memcpy(&v.d, p, 8);
      p += 8;
      break;
    case kTBinary: {
      const uint64_t n = varint();
      if (!ok || n > (uint64_t)(end - p)) {
        ok = false;
        return;
      }
      v.bin.assign((const char*)p, (size_t)n);
      p += n;
      break;
    }
    case kTList:
    case kTSet: {
      const uint8_t h = byte();
      uint64_t n = h >> 4;
      v.etype = h & 0x0F;
      if (n == 15) n = varint();
      if (!ok || n > (uint64_t)(end - p)) {
        ok = false;
        return;
      }
      v.elems.resize((size_t)n);
      for (auto& e : v.elems) {
        if (v.etype == kTTrue || v.etype == kTFalse) {  // booleans in containers: a byte each
          e.type = v.etype;
          e.i = byte() == kTTrue;
        } else {
          value(v.etype, e, depth + 1);
        }
        if (!ok) return;
      }
      break;
    }
    case kTMap: {
      const uint64_t n = varint();
      if (!ok || n > (uint64_t)(end - p)) {
        ok = false;
        return;
      }
      if (n) {
        const uint8_t kv = byte();
        v.etype = kv >> 4;
        v.vtype = kv & 0x0F;
      }
      v.elems.resize((size_t)(2 * n));
      for (size_t k = 0; k < v.elems.size() && ok; ++k) value(k & 1 ? v.vtype : v.etype, v.elems[k], depth + 1);
      break;
    }
    case kTStruct: fields(v.fields, depth); break;
    default: ok = false;
  }
}

struct Writer {
  std::string out;
  void byte(uint8_t b) { out.push_back((char)b); }
  void varint(uint64_t v) {
    while (v >= 0x80) {
      byte((uint8_t)(v | 0x80));
      v >>= 7;
    }
    byte((uint8_t)v);
  }
  void zigzag(int64_t v) { varint(((uint64_t)v << 1) ^ (uint64_t)(v >> 63)); }
  void value(const TVal& v) {
    switch (v.type) {
      case kTTrue:
      case kTFalse: break;  // (in the field header)
      case kTByte: byte((uint8_t)v.i); break;
      case kTI16:
      case kTI32:
      case kTI64: zigzag(v.i); break;
      case kTDouble: out.append((const char*)&v.d, 8); break;
      case kTBinary:
        varint(v.bin.size());
        out.append(v.bin);
        break;
      case kTList:
      case kTSet:
        if (v.elems.size() < 15) {
          byte((uint8_t)(v.elems.size() << 4 | v.etype));
        } else {
          byte((uint8_t)(0xF0 | v.etype));
          varint(v.elems.size());
        }
        for (const auto& e : v.elems) {
          if (v.etype == kTTrue || v.etype == kTFalse) byte(e.i ? kTTrue : kTFalse);
          else value(e);
        }
        break;
      case kTMap:
        varint(v.elems.size() / 2);
        if (!v.elems.empty()) byte((uint8_t)(v.etype << 4 | v.vtype));
        for (const auto& e : v.elems) value(e);
        break;
      case kTStruct: fields(v.fields); break;
    }
  }
  void fields(const std::vector<TField>& fs) {
    int16_t last = 0;
    for (const auto& f : fs) {
      const uint8_t type = (f.v.type == kTTrue || f.v.type == kTFalse) ? (f.v.i ? kTTrue : kTFalse) : f.v.type;
      const int delta = f.id - last;
      if (delta > 0 && delta <= 15) {
        byte((uint8_t)(delta << 4 | type));
      } else {
        byte(type);
        zigzag(f.id);
      }
      value(f.v);
      last = f.id;
    }
    byte(kTStop);
  }
};

TField* field(std::vector<TField>& fs, int16_t id) {
  for (auto& f : fs)
    if (f.id == id) return &f;
  return nullptr;
}
const TField* field(const std::vector<TField>& fs, int16_t id) {
  for (const auto& f : fs)
    if (f.id == id) return &f;
  return nullptr;
}
// set an integer field (kept in field-id order)
void set_int(std::vector<TField>& fs, int16_t id, uint8_t type, int64_t v) {
  if (TField* f = field(fs, id)) {
    f->v.type = type;
    f->v.i = v;
    return;
  }
  TField nf{id, {}};
  nf.v.type = type;
  nf.v.i = v;
  auto it = fs.begin();
  while (it != fs.end() && it->id < id) ++it;
  fs.insert(it, std::move(nf));
}

// ------------------------------------------------------- gzip compressors ----
struct Libdeflate {
  typedef void* (*alloc_fn)(int);
  typedef size_t (*gzip_fn)(void*, const void*, size_t, void*, size_t);
  typedef size_t (*bound_fn)(void*, size_t);
  typedef void (*free_fn)(void*);
  typedef uint32_t (*crc_fn)(uint32_t, const void*, size_t);
  alloc_fn alloc = nullptr;
  gzip_fn gzip = nullptr;
  bound_fn bound = nullptr;
  free_fn free = nullptr;
  crc_fn crc = nullptr;
  static const Libdeflate& get() {
    static const Libdeflate d = [] {
      Libdeflate x;
      void* h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
      if (!h) return x;
      x.alloc = (alloc_fn)dlsym(h, "libdeflate_alloc_compressor");
      x.gzip = (gzip_fn)dlsym(h, "libdeflate_gzip_compress");
      x.bound = (bound_fn)dlsym(h, "libdeflate_gzip_compress_bound");
      x.free = (free_fn)dlsym(h, "libdeflate_free_compressor");
      x.crc = (crc_fn)dlsym(h, "libdeflate_crc32");
      if (!x.alloc || !x.gzip || !x.bound || !x.free || !x.crc) x = Libdeflate{};
      return x;
    }();
    return d;
  }
  bool ok() const { return alloc != nullptr; }
};

uint32_t crc32_of(const uint8_t* p, size_t n) {
  const Libdeflate& L = Libdeflate::get();
  if (L.ok()) return L.crc(0, p, n);
  uLong c = crc32(0L, Z_NULL, 0);
  while (n) {
    const uInt k = (uInt)std::min<size_t>(n, 1u << 30);
    c = crc32(c, p, k);
    p += k;
    n -= k;
  }
  return (uint32_t)c;
}

// gzip member of `n` bytes at `level` (libdeflate, else zlib)
bool gzip_level(const uint8_t* in, size_t n, int level, std::string& out) {
  const Libdeflate& L = Libdeflate::get();
  if (L.ok()) {
    void* c = L.alloc(level);
    if (!c) return false;
    out.resize(L.bound(c, n));
    const size_t k = L.gzip(c, in, n, &out[0], out.size());
    L.free(c);
    out.resize(k);
    return k > 0;
  }
  z_stream zs{};
  if (deflateInit2(&zs, level, Z_DEFLATED, 31, 8, Z_DEFAULT_STRATEGY) != Z_OK) return false;
  out.resize(deflateBound(&zs, (uLong)n) + 32);
  zs.next_in = (Bytef*)in;
  zs.avail_in = (uInt)n;
  zs.next_out = (Bytef*)&out[0];
  zs.avail_out = (uInt)out.size();
  const int rc = deflate(&zs, Z_FINISH);
  out.resize(zs.total_out);
  deflateEnd(&zs);
  return rc == Z_STREAM_END;
}

// LSB-first bit writer (DEFLATE's bit order)
struct Bits {
  std::string& out;
  uint64_t acc = 0;
  int n = 0;
  explicit Bits(std::string& o) : out(o) {}
  void put(uint32_t v, int k) {  // k <= 32
    acc |= (uint64_t)v << n;
    n += k;
    while (n >= 8) {
      out.push_back((char)(acc & 0xFF));
      acc >>= 8;
      n -= 8;
    }
  }
  void flush() {
    if (n > 0) out.push_back((char)(acc & 0xFF));
    acc = 0;
    n = 0;
  }
};

// Length-limited Huffman code lengths (package-free: a Huffman tree, then
// the Kraft-sum repair miniz / zlib use for over-long codes).  freq[i] = 0:
// no code.  At least one symbol must have a non-zero frequency.
void huff_lengths(const uint32_t* freq, int n, int max_len, uint8_t* len) {
  std::vector<int> sym;
  for (int i = 0; i < n; ++i) {
    len[i] = 0;
    if (freq[i]) sym.push_back(i);
  }
  if (sym.size() == 1) {
    len[sym[0]] = 1;
    return;
  }
  std::sort(sym.begin(), sym.end(), [&](int a, int b) { return freq[a] != freq[b] ? freq[a] < freq[b] : a < b; });
  // two-queue Huffman over the sorted leaves; parent links give the depths
  const int m = (int)sym.size();
  std::vector<uint64_t> w(2 * m);
  std::vector<int> parent(2 * m, -1);
  for (int i = 0; i < m; ++i) w[i] = freq[sym[i]];
  int leaf = 0, inner = m, next = m;
  auto pick = [&]() {
    if (leaf < m && (inner >= next || w[leaf] <= w[inner])) return leaf++;
    return inner++;
  };
  for (; next < 2 * m - 1; ++next) {
    const int a = pick(), b = pick();
    w[next] = w[a] + w[b];
    parent[a] = parent[b] = next;
  }
  std::vector<int> depth(2 * m, 0);
  for (int i = 2 * m - 3; i >= 0; --i) depth[i] = depth[parent[i]] + 1;
  // code-length counts, then the repair for lengths over max_len
  std::vector<int> count(64, 0);
  for (int i = 0; i < m; ++i) count[std::min(depth[i], 63)]++;
  for (int k = max_len + 1; k < 64; ++k) {
    count[max_len] += count[k];
    count[k] = 0;
  }
  uint64_t total = 0;
  for (int k = max_len; k > 0; --k) total += (uint64_t)count[k] << (max_len - k);
  while (total > (1ull << max_len)) {
    count[max_len]--;
    for (int k = max_len - 1; k > 0; --k)
      if (count[k]) {
        count[k]--;
        count[k + 1] += 2;
        break;
      }
    total--;
  }
  // the shortest codes to the most frequent symbols
  int k = max_len, left = count[max_len];
  for (int i = 0; i < m; ++i) {  // sym ascending by frequency: longest codes first
    while (left == 0) left = count[--k];
    len[sym[i]] = (uint8_t)k;
    --left;
  }
}
// canonical codes, bit-reversed for the LSB-first stream
void huff_codes(const uint8_t* len, int n, uint32_t* code) {
  int bl_count[16] = {0}, next_code[16] = {0};
  for (int i = 0; i < n; ++i) bl_count[len[i]]++;
  bl_count[0] = 0;
  int c = 0;
  for (int b = 1; b < 16; ++b) {
    c = (c + bl_count[b - 1]) << 1;
    next_code[b] = c;
  }
  for (int i = 0; i < n; ++i) {
    code[i] = 0;
    if (!len[i]) continue;
    uint32_t v = (uint32_t)next_code[len[i]]++, r = 0;
    for (int b = 0; b < len[i]; ++b) r |= ((v >> b) & 1u) << (len[i] - 1 - b);
    code[i] = r;
  }
}

// one gzip member holding one dynamic-Huffman DEFLATE block of the bytes as
// literals (RFC 1951 §3.2.7; RFC 1952)
void gzip_huffman(const uint8_t* in, size_t n, std::string& out) {
  uint32_t freq[257] = {0};
  {
    uint32_t f4[4][256] = {{0}};  // four tables: no store-to-load chain on runs of one byte
    size_t i = 0;
    for (; i + 4 <= n; i += 4) {
      f4[0][in[i]]++;
      f4[1][in[i + 1]]++;
      f4[2][in[i + 2]]++;
      f4[3][in[i + 3]]++;
    }
    for (; i < n; ++i) f4[0][in[i]]++;
    for (int s = 0; s < 256; ++s) freq[s] = f4[0][s] + f4[1][s] + f4[2][s] + f4[3][s];
  }
  freq[256] = 1;  // end of block
  uint8_t len[258];
  huff_lengths(freq, 257, 15, len);
  len[257] = 0;  // the one distance code: length 0, none used (all literals)
  uint32_t code[257];
  huff_codes(len, 257, code);
  // the 258 code lengths, run-length coded with the code-length alphabet:
  // 0..15 literal, 17 = 3..10 zeros, 18 = 11..138 zeros
  std::vector<std::pair<int, int>> cl;  // (symbol, extra)
  for (int i = 0; i < 258;) {
    if (len[i] == 0) {
      int j = i;
      while (j < 258 && len[j] == 0 && j - i < 138) ++j;
      const int r = j - i;
      if (r >= 11) cl.push_back({18, r - 11});
      else if (r >= 3) cl.push_back({17, r - 3});
      else
        for (int k = 0; k < r; ++k) cl.push_back({0, 0});
      i = j;
    } else {
      cl.push_back({len[i], 0});
      ++i;
    }
  }
  uint32_t cfreq[19] = {0};
  for (const auto& s : cl) cfreq[s.first]++;
  uint8_t clen[19];
  huff_lengths(cfreq, 19, 7, clen);
  uint32_t ccode[19];
  huff_codes(clen, 19, ccode);
  static const int kOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
  int hclen = 19;
  while (hclen > 4 && clen[kOrder[hclen - 1]] == 0) --hclen;

  out.clear();
  out.reserve(n / 2 + 256);
  static const uint8_t kHdr[10] = {0x1f, 0x8b, 8, 0, 0, 0, 0, 0, 0, 3};  // no flags, no mtime, unix
  out.append((const char*)kHdr, 10);
  Bits b(out);
  b.put(1, 1);  // BFINAL
  b.put(2, 2);  // BTYPE = dynamic Huffman
  b.put(257 - 257, 5);  // HLIT
  b.put(1 - 1, 5);      // HDIST
  b.put((uint32_t)(hclen - 4), 4);
  for (int i = 0; i < hclen; ++i) b.put(clen[kOrder[i]], 3);
  for (const auto& s : cl) {
    b.put(ccode[s.first], clen[s.first]);
    if (s.first == 17) b.put((uint32_t)s.second, 3);
    if (s.first == 18) b.put((uint32_t)s.second, 7);
  }
  // the literals: two bytes a step (<= 30 bits) into a 64-bit accumulator
  // holding < 32 bits, a 32-bit word stored every step and kept when full
  // (no data-dependent branch)
  uint32_t ent[256];
  for (int s = 0; s < 256; ++s) ent[s] = code[s] | (uint32_t)len[s] << 16;
  uint64_t acc = b.acc;
  uint32_t nb = (uint32_t)b.n;
  const size_t base = out.size();
  out.resize(base + n * 2 + 16);  // (<= 15 bits a byte)
  uint8_t* o = (uint8_t*)&out[base];
  size_t w = 0, i = 0;
  for (; i + 2 <= n; i += 2) {
    const uint32_t e0 = ent[in[i]], e1 = ent[in[i + 1]];
    const uint32_t l0 = e0 >> 16;
    const uint64_t v = (uint64_t)(e0 & 0xFFFFu) | (uint64_t)(e1 & 0xFFFFu) << l0;
    acc |= v << nb;
    nb += l0 + (e1 >> 16);
    const uint32_t lo = (uint32_t)acc;
    memcpy(o + w, &lo, 4);
    const uint32_t f = nb >> 5;  // 0 or 1
    w += 4 * f;
    acc >>= 32 * f;
    nb -= 32 * f;
  }
  for (; i < n; ++i) {
    const uint32_t e = ent[in[i]];
    acc |= (uint64_t)(e & 0xFFFFu) << nb;
    nb += e >> 16;
    if (nb >= 32) {
      const uint32_t lo = (uint32_t)acc;
      memcpy(o + w, &lo, 4);
      w += 4;
      acc >>= 32;
      nb -= 32;
    }
  }
  out.resize(base + w);
  b.acc = acc;
  b.n = (int)nb;
  b.put(code[256], len[256]);  // end of block
  b.flush();
  const uint32_t crc = crc32_of(in, n), isize = (uint32_t)n;
  out.append((const char*)&crc, 4);
  out.append((const char*)&isize, 4);
}

// ------------------------------------------------------------- the file ----
constexpr int64_t kCodecGzip = 2;
enum : int32_t { kPageData = 0, kPageIndex = 1, kPageDict = 2, kPageDataV2 = 3 };

struct Page {
  int64_t hdr_pos = 0, data_pos = 0, data_len = 0;
  std::vector<TField> hdr;
  bool huff = false;
  std::string body, hdr_out;  // compressed page, re-encoded header
};
struct Chunk {
  TVal* cc;  // the ColumnChunk struct in the footer tree
  int64_t start = 0, len = 0;
  std::vector<Page> pages;
  bool huff = false;
};

bqsr_status rewrite(const uint8_t* in, int64_t n, const char* path, int level, const char* huffman_cols,
                    int threads, int64_t* out_len) {
  auto bad = [](const std::string& m) { return fail(BQSR_ERR_INVALID_ARG, "bqsr_parquet_gzip: " + m); };
  if (n < 12 || memcmp(in, "PAR1", 4) != 0 || memcmp(in + n - 4, "PAR1", 4) != 0) return bad("not a Parquet file");
  uint32_t flen;
  memcpy(&flen, in + n - 8, 4);
  if ((int64_t)flen + 12 > n) return bad("footer length");
  const uint8_t* fp = in + n - 8 - flen;
  Reader fr{fp, fp + flen};
  TVal meta;
  meta.type = kTStruct;
  fr.fields(meta.fields, 0);
  if (!fr.ok) return bad("footer does not parse");
  std::vector<std::string> hcols;
  for (const char* s = huffman_cols ? huffman_cols : ""; *s;) {
    const char* e = strchr(s, ',');
    hcols.emplace_back(s, e ? (size_t)(e - s) : strlen(s));
    s = e ? e + 1 : s + strlen(s);
  }
  TField* rgs = field(meta.fields, 4);
  std::vector<Chunk> chunks;
  if (rgs) {
    for (auto& rg : rgs->v.elems) {
      TField* cols = field(rg.fields, 1);
      if (!cols) return bad("row group without columns");
      for (auto& cc : cols->v.elems) {
        TField* md = field(cc.fields, 3);
        if (!md || field(cc.fields, 1) || field(cc.fields, 4) || field(cc.fields, 6))
          return bad("column chunk layout not supported (external file, page index)");
        auto& m = md->v.fields;
        const TField* codec = field(m, 4);
        if (!codec || codec->v.i != 0) return bad("input pages must be uncompressed");
        if (field(m, 10) || field(m, 14)) return bad("index pages / bloom filters not supported");
        const TField* dpo = field(m, 9);
        const TField* dic = field(m, 11);
        const TField* tcs = field(m, 7);
        if (!dpo || !tcs) return bad("column chunk without offsets");
        Chunk c;
        c.cc = &cc;
        // (a chunk without rows has a dictionary page and data_page_offset 0)
        const int64_t d0 = dic && dic->v.i > 0 ? dic->v.i : -1, p0 = dpo->v.i > 0 ? dpo->v.i : -1;
        c.start = d0 < 0 ? p0 : p0 < 0 ? d0 : std::min(d0, p0);
        c.len = tcs->v.i;
        if (c.len == 0) c.start = 4;  // (a chunk without pages: a boolean column of no rows)
        if (c.start < 4 || c.len < 0 || c.start + c.len > n - 8 - (int64_t)flen) return bad("chunk out of range");
        const TField* path = field(m, 3);
        if (path && !path->v.elems.empty())
          for (const auto& h : hcols) c.huff |= path->v.elems[0].bin == h;
        chunks.push_back(c);
      }
    }
  }
  // the pages of every chunk
  for (auto& c : chunks) {
    int64_t pos = c.start;
    while (pos < c.start + c.len) {
      Page pg;
      pg.hdr_pos = pos;
      Reader r{in + pos, in + c.start + c.len};
      r.fields(pg.hdr, 0);
      if (!r.ok) return bad("page header does not parse");
      const TField* t = field(pg.hdr, 1);
      const TField* us = field(pg.hdr, 2);
      const TField* cs = field(pg.hdr, 3);
      if (!t || !us || !cs || us->v.i != cs->v.i) return bad("page sizes");
      if (t->v.i == kPageDataV2 || t->v.i == kPageIndex) return bad("data page v2 / index pages not supported");
      pg.data_pos = (int64_t)(r.p - in);
      pg.data_len = cs->v.i;
      if (pg.data_pos + pg.data_len > c.start + c.len) return bad("page out of range");
      pg.huff = c.huff;
      pos = pg.data_pos + pg.data_len;
      c.pages.push_back(std::move(pg));
    }
  }
  // compress every page (threads over all pages of the file)
  std::vector<Page*> all;
  for (auto& c : chunks)
    for (auto& p : c.pages) all.push_back(&p);
  std::atomic<size_t> next{0};
  std::atomic<bool> okc{true};
  auto work_pages = [&]() {
    for (size_t i; okc && (i = next.fetch_add(1)) < all.size();) {
      Page& p = *all[i];
      const uint8_t* d = in + p.data_pos;
      if (p.huff) gzip_huffman(d, (size_t)p.data_len, p.body);
      else if (!gzip_level(d, (size_t)p.data_len, level, p.body)) okc = false;
      set_int(p.hdr, 3, kTI32, (int64_t)p.body.size());
      if (field(p.hdr, 4)) set_int(p.hdr, 4, kTI32, (int32_t)crc32_of((const uint8_t*)p.body.data(), p.body.size()));
      Writer w;
      w.fields(p.hdr);
      p.hdr_out = std::move(w.out);
    }
  };
  // (a worker's exception -- std::bad_alloc from the page buffers -- must not
  // escape its thread, which would std::terminate the process: it fails the
  // call after the join instead)
  auto work = [&]() {
    try {
      work_pages();
    } catch (...) {
      okc = false;
    }
  };
  const int nt = std::max(1, std::min<int>(threads, (int)all.size()));
  std::vector<std::thread> pool;
  for (int t = 1; t < nt; ++t) pool.emplace_back(work);
  work();
  for (auto& t : pool) t.join();
  if (!okc) return fail(BQSR_ERR_DEVICE, "bqsr_parquet_gzip: compression failed");
  // the new layout: chunks in file order, their pages back to back
  std::sort(chunks.begin(), chunks.end(), [](const Chunk& a, const Chunk& b) { return a.start < b.start; });
  std::vector<std::pair<int64_t, int64_t>> moved;  // old page offset -> new
  int64_t pos = 4;
  for (auto& c : chunks) {
    TField* md = field(c.cc->fields, 3);
    auto& m = md->v.fields;
    const int64_t old_start = c.start;
    int64_t tcs = 0, tus = 0, dict_new = -1, data_new = -1;
    for (const auto& p : c.pages) {
      moved.push_back({p.hdr_pos, pos});
      const TField* t = field(p.hdr, 1);
      if (t->v.i == kPageDict && dict_new < 0) dict_new = pos;
      if (t->v.i == kPageData && data_new < 0) data_new = pos;
      tcs += (int64_t)(p.hdr_out.size() + p.body.size());
      tus += (int64_t)p.hdr_out.size() + p.data_len;
      pos += (int64_t)(p.hdr_out.size() + p.body.size());
    }
    moved.push_back({old_start + c.len, pos});  // (an offset at the chunk's end: its new end)
    set_int(m, 4, kTI32, kCodecGzip);
    set_int(m, 6, kTI64, tus);
    set_int(m, 7, kTI64, tcs);
    if (data_new >= 0) set_int(m, 9, kTI64, data_new);
    if (field(m, 11) && dict_new >= 0) set_int(m, 11, kTI64, dict_new);
    c.start = old_start;
  }
  auto map_off = [&](int64_t old) -> int64_t {
    for (const auto& mv : moved)
      if (mv.first == old) return mv.second;
    return old;  // (an offset not at a page: left as it was)
  };
  if (rgs) {
    for (auto& rg : rgs->v.elems) {
      int64_t tcs = 0;
      for (auto& cc : field(rg.fields, 1)->v.elems) {
        if (TField* fo = field(cc.fields, 2)) fo->v.i = map_off(fo->v.i);
        tcs += field(field(cc.fields, 3)->v.fields, 7)->v.i;
      }
      if (TField* fo = field(rg.fields, 5)) fo->v.i = map_off(fo->v.i);
      if (field(rg.fields, 6)) set_int(rg.fields, 6, kTI64, tcs);
    }
  }
  Writer fw;
  fw.fields(meta.fields);
  // write the file
  FILE* f = fopen(path, "wb");
  if (!f) return fail(BQSR_ERR_INVALID_ARG, std::string("bqsr_parquet_gzip: cannot open ") + path);
  bool wok = fwrite("PAR1", 1, 4, f) == 4;
  for (const auto& c : chunks)
    for (const auto& p : c.pages) {
      wok = wok && fwrite(p.hdr_out.data(), 1, p.hdr_out.size(), f) == p.hdr_out.size();
      wok = wok && fwrite(p.body.data(), 1, p.body.size(), f) == p.body.size();
    }
  const uint32_t fl = (uint32_t)fw.out.size();
  wok = wok && fwrite(fw.out.data(), 1, fw.out.size(), f) == fw.out.size();
  wok = wok && fwrite(&fl, 1, 4, f) == 4 && fwrite("PAR1", 1, 4, f) == 4;
  wok = fclose(f) == 0 && wok;
  if (!wok) return fail(BQSR_ERR_DEVICE, std::string("bqsr_parquet_gzip: write failed: ") + path);
  if (out_len) *out_len = pos + (int64_t)fw.out.size() + 8;
  return BQSR_OK;
}

}  // namespace pqgz

extern "C" bqsr_status bqsr_parquet_gzip(const uint8_t* in, int64_t in_len, const char* path, int32_t level,
                                         const char* huffman_cols, int32_t threads, int64_t* out_len) {
  if (!in || !path || in_len < 0 || level < 0 || level > 12)
    return fail(BQSR_ERR_INVALID_ARG, "bqsr_parquet_gzip: bad arguments");
  try {
    const bqsr_status st = pqgz::rewrite(in, in_len, path, level, huffman_cols, threads, out_len);
    if (st == BQSR_OK) ok();
    return st;
  } catch (const std::bad_alloc&) {
    return fail(BQSR_ERR_DEVICE, "bqsr_parquet_gzip: out of host memory");
  }
}

// one page's worth of bytes through the two compressors (tests)
extern "C" bqsr_status bqsr_gzip_bytes(const uint8_t* in, int64_t n, int32_t huffman, int32_t level, uint8_t* out,
                                       int64_t cap, int64_t* out_len) {
  if ((!in && n) || n < 0 || !out_len) return fail(BQSR_ERR_INVALID_ARG, "bqsr_gzip_bytes: bad arguments");
  std::string s;
  if (huffman) pqgz::gzip_huffman(in, (size_t)n, s);
  else if (!pqgz::gzip_level(in, (size_t)n, level, s)) return fail(BQSR_ERR_DEVICE, "bqsr_gzip_bytes: failed");
  *out_len = (int64_t)s.size();
  if (out && cap >= (int64_t)s.size()) memcpy(out, s.data(), s.size());
  return ok();
}
