// synth.cpp -- deterministic synthetic ADAMRecord partitions.
//
// Host-only C++ (g++), multi-threaded; every read is generated from its own
// counter-based RNG stream (seed, read index), so a read is the same whatever
// the thread split and the output is reproducible across machines.
//
//   bases : uniform ACGT, 0.1 % N
//   quals : clamp(round(N(38 - 10 (o/L)^2, 3)), 3, 41); 1 % of reads end in a
//           Q2 run of 1-10 bases (exercises quality trimming)
//   error : Bernoulli(10^(-(q-2)/10)) per aligned base -> MD mismatch
//   CIGAR : 95 % LM; 3 % one 1-3 bp I or D; 2 % a 1-20 bp soft clip
//   flags : paired, 50 % second of pair, 50 % reverse strand,
//           1 % unmapped, 1 % duplicate, 0.5 % secondary
//   start : uniform on the contig
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace {

struct Rng {  // splitmix64 stream
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed) {}
  uint64_t next() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  double uni() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
  uint32_t below(uint32_t n) { return (uint32_t)(uni() * n); }
  // Box-Muller, both outputs used
  bool have = false;
  double spare = 0.0;
  double normal() {
    if (have) {
      have = false;
      return spare;
    }
    double u1 = uni(), u2 = uni();
    if (u1 < 1e-300) u1 = 1e-300;
    const double r = std::sqrt(-2.0 * std::log(u1));
    spare = r * std::sin(6.283185307179586 * u2);
    have = true;
    return r * std::cos(6.283185307179586 * u2);
  }
};

}  // namespace

extern "C" {

struct SynthSpec {
  int64_t n_reads;
  uint64_t seed;
  int32_t n_len;          // number of read-length choices
  const int32_t* lens;    // [n_len], chosen uniformly
  int32_t n_rg;           // read groups, chosen uniformly
  int64_t contig_len;
  double p_unmapped, p_duplicate, p_secondary, p_n, p_q2tail, p_indel, p_softclip;
  int64_t first_read;     // index of read 0 in the whole dataset: reads [first, first + n) of one
                          // (seed, ...) dataset, so a rank's shard is a slice of the job's reads
  int64_t sorted_total;   // > 0: coordinate-sorted (what `transform -sort_reads` leaves): read i of the
                          // sorted_total-read dataset starts at i / sorted_total of the contig
};

// flag bits as include/adam_bqsr.h
enum : uint32_t {
  F_PAIRED = 1u << 0, F_MAPPED = 1u << 1, F_NEG = 1u << 2, F_SECOND = 1u << 3, F_PRIMARY = 1u << 4,
  F_DUP = 1u << 5, F_HAS_RG = 1u << 8, F_HAS_MD = 1u << 9, F_HAS_QUAL = 1u << 10, F_HAS_SEQ = 1u << 11,
  F_HAS_CIGAR = 1u << 12, F_HAS_START = 1u << 13, F_HAS_REFNAME = 1u << 14
};

}  // extern "C"

namespace {

struct Read {
  uint32_t flags = 0;
  int32_t rg = 0;
  int64_t start = 0;
  std::string seq, qual, md;
  std::vector<uint32_t> cigar;
};

const char kBases[4] = {'A', 'C', 'G', 'T'};

struct ErrTab {  // Bernoulli(10^(-(q-2)/10)) per qual
  double p[64];
  ErrTab() {
    for (int q = 0; q < 64; ++q) p[q] = std::min(1.0, std::pow(10.0, -(q - 2) / 10.0));
  }
} const kErr;

void append_int(std::string& s, int v) {
  char b[12];
  int n = 0;
  do {
    b[n++] = (char)('0' + v % 10);
    v /= 10;
  } while (v);
  while (n) s += b[--n];
}

void gen_read(const SynthSpec& sp, int64_t r, Read& R) {
  r += sp.first_read;
  Rng g(sp.seed * 0x9E3779B97F4A7C15ull ^ (uint64_t)r * 0xD1B54A32D192ED03ull ^ 0x5851F42D4C957F2Dull);
  g.next();
  const int L = sp.lens[sp.n_len > 1 ? g.below((uint32_t)sp.n_len) : 0];
  R.rg = sp.n_rg > 1 ? (int32_t)g.below((uint32_t)sp.n_rg) : 0;
  uint32_t f = F_PAIRED | F_HAS_RG | F_HAS_QUAL | F_HAS_SEQ | F_HAS_CIGAR;
  if (g.uni() < 0.5) f |= F_SECOND;
  if (g.uni() < 0.5) f |= F_NEG;
  const bool unmapped = g.uni() < sp.p_unmapped;
  if (g.uni() >= sp.p_secondary) f |= F_PRIMARY;
  if (g.uni() < sp.p_duplicate) f |= F_DUP;
  // bases
  R.seq.resize((size_t)L);
  for (int i = 0; i < L; ++i) R.seq[(size_t)i] = g.uni() < sp.p_n ? 'N' : kBases[g.below(4)];
  // quals
  std::vector<int> q((size_t)L);
  for (int i = 0; i < L; ++i) {
    const double x = (double)i / L;
    long v = std::lround(38.0 - 10.0 * x * x + 3.0 * g.normal());
    q[(size_t)i] = (int)std::min(41L, std::max(3L, v));
  }
  if (g.uni() < sp.p_q2tail) {
    const int k = 1 + (int)g.below(10);
    for (int i = std::max(0, L - k); i < L; ++i) q[(size_t)i] = 2;
  }
  R.qual.resize((size_t)L);
  for (int i = 0; i < L; ++i) R.qual[(size_t)i] = (char)(q[(size_t)i] + 33);
  // alignment
  R.cigar.clear();
  R.md.clear();
  if (unmapped) {
    R.flags = f;  // no MAPPED / MD / start / referenceName; CIGAR "*"
    R.start = 0;
    return;
  }
  f |= F_MAPPED | F_HAS_MD | F_HAS_START | F_HAS_REFNAME;
  const double u = g.uni();
  int lead_s = 0, trail_s = 0, ins_at = -1, ins_len = 0, del_at = -1, del_len = 0;
  if (u < sp.p_indel && L > 24) {
    const int at = 10 + (int)g.below((uint32_t)(L - 20));
    const int len = 1 + (int)g.below(3);
    if (g.uni() < 0.5) {
      ins_at = at;
      ins_len = len;
    } else {
      del_at = at;
      del_len = len;
    }
  } else if (u < sp.p_indel + sp.p_softclip && L > 24) {
    const int len = 1 + (int)g.below(20);
    if (g.uni() < 0.5) lead_s = len; else trail_s = len;
  }
  auto push = [&](int len, uint32_t op) {
    if (len > 0) R.cigar.push_back(((uint32_t)len << 4) | op);
  };
  // ops: S=4 M=0 I=1 D=2
  if (ins_at >= 0) {
    push(ins_at, 0);
    push(ins_len, 1);
    push(L - ins_at - ins_len, 0);
  } else if (del_at >= 0) {
    push(del_at, 0);
    push(del_len, 2);
    push(L - del_at, 0);
  } else {
    push(lead_s, 4);
    push(L - lead_s - trail_s, 0);
    push(trail_s, 4);
  }
  int64_t span = 0;
  for (uint32_t e : R.cigar)
    if ((e & 0xF) == 0 || (e & 0xF) == 2) span += e >> 4;
  const double u_start = g.uni();
  R.start = sp.sorted_total > 0
                ? (int64_t)((double)r / (double)sp.sorted_total * (double)std::max<int64_t>(1, sp.contig_len - 600))
                : (int64_t)(u_start * (double)std::max<int64_t>(1, sp.contig_len - span - 1));
  // MD over M bases (mismatch = sequencing error) and deletions
  int run = 0;
  int ro = 0;
  for (uint32_t e : R.cigar) {
    const uint32_t op = e & 0xF, len = e >> 4;
    if (op == 4 || op == 1) {  // soft clip / insertion: no reference
      ro += (int)len;
      continue;
    }
    if (op == 2) {
      append_int(R.md, run);
      run = 0;
      R.md += '^';
      for (uint32_t k = 0; k < len; ++k) R.md += kBases[g.below(4)];
      continue;
    }
    for (uint32_t k = 0; k < len; ++k, ++ro) {
      const int qq = q[(size_t)ro];
      const double perr = kErr.p[qq];
      if (g.uni() < perr) {
        append_int(R.md, run);
        run = 0;
        const char rb = R.seq[(size_t)ro];
        int c = rb == 'A' ? 0 : rb == 'C' ? 1 : rb == 'G' ? 2 : rb == 'T' ? 3 : 0;
        R.md += kBases[(c + 1 + g.below(3)) & 3];
      } else {
        ++run;
      }
    }
  }
  append_int(R.md, run);
  R.flags = f;
}

template <class F>
void parallel(int64_t n, int nth, F&& f) {
  std::vector<std::thread> th;
  for (int t = 0; t < nth; ++t) th.emplace_back([&, t] { f(n * t / nth, n * (t + 1) / nth); });
  for (auto& x : th) x.join();
}

}  // namespace

extern "C" {

// Pass 1: per-read sizes -> offsets ([n+1] each; seq and qual share seq_off).
void synth_plan(const SynthSpec* sp, int nthreads, uint64_t* seq_off, uint64_t* cig_off, uint64_t* md_off) {
  const int64_t n = sp->n_reads;
  seq_off[0] = cig_off[0] = md_off[0] = 0;
  parallel(n, nthreads, [&](int64_t a, int64_t b) {
    Read R;
    for (int64_t r = a; r < b; ++r) {
      gen_read(*sp, r, R);
      seq_off[r + 1] = R.seq.size();
      cig_off[r + 1] = R.cigar.size();
      md_off[r + 1] = R.md.size();
    }
  });
  for (int64_t r = 0; r < n; ++r) {
    seq_off[r + 1] += seq_off[r];
    cig_off[r + 1] += cig_off[r];
    md_off[r + 1] += md_off[r];
  }
}

// Pass 2: fill the columns (bqsr_records layout; ref_index 0 = the one contig).
void synth_fill(const SynthSpec* sp, int nthreads, const uint64_t* seq_off, const uint64_t* cig_off,
                const uint64_t* md_off, uint32_t* flags, int32_t* rg, int32_t* ref_index, int64_t* start,
                uint8_t* seq, uint8_t* qual, uint32_t* cigar, uint8_t* md) {
  parallel(sp->n_reads, nthreads, [&](int64_t a, int64_t b) {
    Read R;
    for (int64_t r = a; r < b; ++r) {
      gen_read(*sp, r, R);
      flags[r] = R.flags;
      rg[r] = R.rg;
      ref_index[r] = (R.flags & F_HAS_REFNAME) ? 0 : -1;
      start[r] = R.start;
      memcpy(seq + seq_off[r], R.seq.data(), R.seq.size());
      memcpy(qual + seq_off[r], R.qual.data(), R.qual.size());
      if (!R.cigar.empty()) memcpy(cigar + cig_off[r], R.cigar.data(), R.cigar.size() * 4);
      if (!R.md.empty()) memcpy(md + md_off[r], R.md.data(), R.md.size());
    }
  });
}

}  // extern "C"
