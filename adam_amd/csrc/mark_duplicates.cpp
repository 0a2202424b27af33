// MarkDuplicates (include/adam_sam.h) on the host: the
// drop-in for host columns (bqsr_mark_duplicates, the JNI records case) and
// the fallback of the device path (mark_duplicates.hip).
//
// adam-core/.../rdd/MarkDuplicates.scala:24-111 restated over columns:
//   SingleReadBucket (models/SingleReadBucket.scala:27-37): reads grouped by
//     (recordGroupId, readName), split into primary mapped / secondary mapped
//     / unmapped, each in input order;
//   ReferencePositionPair (models/ReferencePositionPair.scala:27-63): the
//     5' positions (RichADAMRecord.fivePrimePosition, :112-118 -- unclipped
//     start, or unclipped end for reverse reads, :77-109) of the bucket's
//     first two primary reads, the smaller one left;
//   grouping by (left position, library of the bucket's first read), then by
//     right position, and the marking rules of MarkDuplicates.apply /
//     markReads / scoreAndMarkReads.
// Buckets keep first-appearance order (Spark's groupBy order is that of its
// shuffle); scoreAndMarkReads' sortBy is stable.
// Included by bqsr_capi.cpp after sam_ingest.hip.

#include <unordered_map>

namespace mdup {

// ReferencePositionWithOrientation of a mapped read (refPos always defined)
struct RPos {
  int32_t ref;
  int64_t pos;
  bool neg;
  bool operator<(const RPos& o) const {
    if (ref != o.ref) return ref < o.ref;
    if (pos != o.pos) return pos < o.pos;
    return !neg && o.neg;  // false < true
  }
  bool operator==(const RPos& o) const { return ref == o.ref && pos == o.pos && neg == o.neg; }
};
struct OptPos {
  bool some = false;
  RPos p{0, 0, false};
  bool operator<(const OptPos& o) const {  // None < Some
    if (some != o.some) return !some;
    return some && p < o.p;
  }
  bool operator==(const OptPos& o) const { return some == o.some && (!some || p == o.p); }
};

struct Bucket {
  std::vector<int64_t> prim, sec, unm;
  OptPos left, right;
  bool has_lib = false;
  std::string lib;
};

// RichADAMRecord.fivePrimePosition
int64_t five_prime(const bqsr_dup_reads& R, int64_t r) {
  const uint32_t* c = R.cigar + R.cigar_offset[r];
  const int64_t n = (int64_t)(R.cigar_offset[r + 1] - R.cigar_offset[r]);
  auto clipped = [](uint32_t e) {
    const uint32_t op = e & 0xF;
    return op == BQSR_CIGAR_S || op == BQSR_CIGAR_H;
  };
  const int64_t start = R.start[r];
  if (!(R.flags[r] & BQSR_F_NEG_STRAND)) {  // unclippedStart
    int64_t p = start;
    for (int64_t i = 0; i < n && clipped(c[i]); ++i) p -= (int64_t)(c[i] >> 4);
    return p;
  }
  int64_t end = start;  // end: + every element consuming reference bases (M D N = X)
  for (int64_t i = 0; i < n; ++i) {
    const uint32_t op = c[i] & 0xF;
    if (op == BQSR_CIGAR_M || op == BQSR_CIGAR_D || op == BQSR_CIGAR_N || op == BQSR_CIGAR_EQ || op == BQSR_CIGAR_X)
      end += (int64_t)(c[i] >> 4);
  }
  for (int64_t i = n - 1; i >= 0 && clipped(c[i]); --i) end += (int64_t)(c[i] >> 4);  // unclippedEnd
  return end;
}

RPos rpos(const bqsr_dup_reads& R, int64_t r) {
  return RPos{R.reference_id[r], five_prime(R, r), (R.flags[r] & BQSR_F_NEG_STRAND) != 0};
}

// MarkDuplicates.score: Σ of the phred scores >= 15 ((char - 33).toByte, signed)
int64_t score(const bqsr_dup_reads& R, int64_t r) {
  int64_t s = 0;
  for (uint64_t k = R.qual_offset[r]; k < R.qual_offset[r + 1]; ++k) {
    const int v = (int)(int8_t)(uint8_t)(R.qual[k] - 33);
    if (v >= 15) s += v;
  }
  return s;
}

void mark(const Bucket& b, std::vector<uint8_t>& dup, bool are_dups) {  // markReads
  for (int64_t r : b.prim) dup[(size_t)r] = are_dups;
  for (int64_t r : b.sec) dup[(size_t)r] = are_dups;
  for (int64_t r : b.unm) dup[(size_t)r] = 0;
}

void score_and_mark(const bqsr_dup_reads& R, const std::vector<const Bucket*>& bs, std::vector<uint8_t>& dup) {
  std::vector<std::pair<int64_t, size_t>> sc;
  for (size_t i = 0; i < bs.size(); ++i) {
    int64_t s = 0;
    for (int64_t r : bs[i]->prim) s += score(R, r);
    sc.emplace_back(s, i);
  }
  std::stable_sort(sc.begin(), sc.end(), [](const auto& a, const auto& b) { return a.first > b.first; });
  for (size_t k = 0; k < sc.size(); ++k) {
    const Bucket& b = *bs[sc[k].second];
    for (int64_t r : b.prim) dup[(size_t)r] = k != 0;
    for (int64_t r : b.sec) dup[(size_t)r] = 1;
    for (int64_t r : b.unm) dup[(size_t)r] = 0;
  }
}

}  // namespace mdup

bqsr_status bqsr_mark_duplicates(const bqsr_dup_reads* R, uint8_t* dup_out) {
  if (!R || R->n_reads < 0 || (R->n_reads > 0 && (!dup_out || !R->flags || !R->rg_id || !R->reference_id ||
                                                  !R->start || !R->qual_offset || !R->cigar_offset)))
    return fail(BQSR_ERR_INVALID_ARG, "bqsr_mark_duplicates: bad arguments");
  using namespace mdup;
  const int64_t n = R->n_reads;
  // ---- SingleReadBucket: group by (recordGroupId, readName) ----
  std::vector<Bucket> buckets;
  {
    std::unordered_map<std::string, size_t> idx;
    std::string key;
    for (int64_t r = 0; r < n; ++r) {
      key.clear();
      if (R->flags[r] & BQSR_F_HAS_RG) key += "g" + std::to_string(R->rg_id[r]);
      else key += "n";
      key.push_back('\0');
      const char* nm = R->read_name ? R->read_name[r] : nullptr;
      if (nm) {
        key.push_back('s');
        key += nm;
      } else {
        key.push_back('n');
      }
      auto it = idx.find(key);
      size_t b;
      if (it == idx.end()) {
        b = buckets.size();
        idx.emplace(key, b);
        buckets.emplace_back();
      } else {
        b = it->second;
      }
      const uint32_t f = R->flags[r];
      if (!(f & BQSR_F_MAPPED)) buckets[b].unm.push_back(r);
      else if (f & BQSR_F_PRIMARY) buckets[b].prim.push_back(r);
      else buckets[b].sec.push_back(r);
    }
  }
  // ---- ReferencePositionPair and the bucket's library ----
  for (Bucket& b : buckets) {
    if (!b.prim.empty()) {
      const RPos p1 = rpos(*R, b.prim[0]);
      if (b.prim.size() > 1) {  // paired with a mapped mate or not: the first two primary reads, ordered
        const RPos p2 = rpos(*R, b.prim[1]);
        b.left.some = b.right.some = true;
        if (p1 < p2) {
          b.left.p = p1;
          b.right.p = p2;
        } else {
          b.left.p = p2;
          b.right.p = p1;
        }
      } else {
        b.left.some = true;
        b.left.p = p1;
      }
    }
    const int64_t r0 = !b.prim.empty() ? b.prim[0] : (!b.sec.empty() ? b.sec[0] : b.unm[0]);  // allReads(0)
    const char* lib = R->library ? R->library[r0] : nullptr;
    b.has_lib = lib != nullptr;
    if (lib) b.lib = lib;
  }
  // ---- group by (left position, library), then by right position ----
  std::vector<uint8_t> dup((size_t)n, 0);
  std::vector<size_t> order(buckets.size());
  for (size_t i = 0; i < order.size(); ++i) order[i] = i;
  auto lib_less = [](const Bucket& a, const Bucket& b) {
    if (a.has_lib != b.has_lib) return !a.has_lib;
    return a.has_lib && a.lib < b.lib;
  };
  auto lib_eq = [](const Bucket& a, const Bucket& b) { return a.has_lib == b.has_lib && (!a.has_lib || a.lib == b.lib); };
  std::stable_sort(order.begin(), order.end(), [&](size_t x, size_t y) {
    const Bucket &a = buckets[x], &b = buckets[y];
    if (!(a.left == b.left)) return a.left < b.left;
    if (!lib_eq(a, b)) return lib_less(a, b);
    return a.right < b.right;  // stable: first appearance inside a group
  });
  size_t i = 0;
  while (i < order.size()) {
    size_t j = i;
    while (j < order.size() && buckets[order[j]].left == buckets[order[i]].left &&
           lib_eq(buckets[order[j]], buckets[order[i]]))
      ++j;
    // group [i, j): one (left, library)
    if (!buckets[order[i]].left.some) {  // unmapped: never duplicates
      for (size_t k = i; k < j; ++k) mark(buckets[order[k]], dup, false);
    } else {
      std::vector<const Bucket*> frags;
      bool has_pairs = false;
      for (size_t k = i; k < j; ++k) {
        if (buckets[order[k]].right.some) has_pairs = true;
        else frags.push_back(&buckets[order[k]]);
      }
      if (has_pairs) {
        for (const Bucket* b : frags) mark(*b, dup, true);  // fragments beside pairs
        size_t k = i;
        while (k < j) {
          if (!buckets[order[k]].right.some) {
            ++k;
            continue;
          }
          size_t m = k;
          std::vector<const Bucket*> g;
          while (m < j && buckets[order[m]].right == buckets[order[k]].right) g.push_back(&buckets[order[m++]]);
          score_and_mark(*R, g, dup);
          k = m;
        }
      } else {
        score_and_mark(*R, frags, dup);
      }
    }
    i = j;
  }
  std::memcpy(dup_out, dup.data(), (size_t)n);
  return ok();
}

namespace {
// the host path of bqsr_sam_mark_duplicates (mark_duplicates.hip's fallback):
// the columns copied back, bqsr_mark_duplicates, FLAG copied up
bqsr_status mark_duplicates_host(bqsr_sam* s, int64_t* n_duplicates) {
  HIP_TRY(hipSetDevice(s->ctx->device));
  const size_t n = (size_t)s->n_reads;
  std::vector<uint32_t> flags(n), raw(n);
  std::vector<int32_t> rg(n), sq(n);
  std::vector<int64_t> start(n);
  std::vector<uint64_t> qo(n + 1), co(n + 1), span(2 * n);
  std::vector<uint8_t> qual((size_t)s->qual_bytes);
  std::vector<uint32_t> cig((size_t)s->cig_ops);
  std::vector<char> text((size_t)s->n_text);
  auto cp = [](void* d, const void* src, size_t b) { return b ? hipMemcpy(d, src, b, hipMemcpyDeviceToHost) : hipSuccess; };
  hipError_t e = cp(flags.data(), s->flags, n * 4);
  if (e == hipSuccess) e = cp(raw.data(), s->raw_flag, n * 4);
  if (e == hipSuccess) e = cp(rg.data(), s->rg_id, n * 4);
  if (e == hipSuccess) e = cp(sq.data(), s->sq_id, n * 4);
  if (e == hipSuccess) e = cp(start.data(), s->start, n * 8);
  if (e == hipSuccess) e = cp(qo.data(), s->qual_off, (n + 1) * 8);
  if (e == hipSuccess) e = cp(co.data(), s->cig_off, (n + 1) * 8);
  if (e == hipSuccess) e = cp(qual.data(), s->qual, qual.size());
  if (e == hipSuccess) e = cp(cig.data(), s->cig, cig.size() * 4);
  if (e == hipSuccess) e = cp(span.data(), s->line_span, 2 * n * 8);
  if (e == hipSuccess) e = cp(text.data(), s->d_text, text.size());
  if (e != hipSuccess) return fail(BQSR_ERR_DEVICE, std::string("bqsr_sam_mark_duplicates: ") + hipGetErrorString(e));
  // readName = QNAME, library = LB of the read group, mateMapped (SAMRecordConverter.scala:72-82)
  std::vector<std::string> names(n);
  std::vector<const char*> name_p(n), lib_p(n);
  std::vector<uint8_t> mate(n);
  for (size_t r = 0; r < n; ++r) {
    const char* a = text.data() + span[2 * r];
    const char* b = (const char*)memchr(a, '\t', (size_t)(span[2 * r + 1] - span[2 * r]));
    names[r].assign(a, b ? (size_t)(b - a) : (size_t)(span[2 * r + 1] - span[2 * r]));
    name_p[r] = names[r].c_str();
    const bool has_rg = flags[r] & BQSR_F_HAS_RG;
    lib_p[r] = (has_rg && (size_t)rg[r] < s->rg_has_lb.size() && s->rg_has_lb[(size_t)rg[r]])
                   ? s->rg_library[(size_t)rg[r]].c_str()
                   : nullptr;
    mate[r] = raw[r] != 0 && (raw[r] & 0x1) && !(raw[r] & 0x8);
  }
  bqsr_dup_reads R{(int64_t)n, name_p.data(), lib_p.data(), flags.data(), mate.data(), rg.data(), sq.data(),
                   start.data(), qo.data(), qual.data(), co.data(), cig.data()};
  std::vector<uint8_t> dup(n);
  bqsr_status st = bqsr_mark_duplicates(&R, dup.data());
  if (st != BQSR_OK) return st;
  int64_t nd = 0;
  for (size_t r = 0; r < n; ++r) {
    flags[r] = dup[r] ? (flags[r] | BQSR_F_DUPLICATE) : (flags[r] & ~(uint32_t)BQSR_F_DUPLICATE);
    nd += dup[r];
  }
  if (n) HIP_TRY(hipMemcpy(s->flags, flags.data(), n * 4, hipMemcpyHostToDevice));
  s->dup_marked = true;
  if (n_duplicates) *n_duplicates = nd;
  return ok();
}
}  // namespace

#include "mark_duplicates.hip"
