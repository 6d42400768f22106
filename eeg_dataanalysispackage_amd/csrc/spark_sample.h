// spark_sample.h -- Spark 1.6.2's RDD.sample(withReplacement = false, fraction, seed) over a
// ParallelCollectionRDD of n rows in N partitions, restated on the host: the mini-batch of
// GradientDescent.runMiniBatchSGD's iteration i is data.sample(false, miniBatchFraction, 42 + i)
// (MLlib 1.6.2, behind LogisticRegressionClassifier.java:98-108 / README.md:136's
// config_mini_batch_fraction).  The CPU restatement the tests check this against is
// oracle/mllib_logreg.py (sample_rows); the algorithm, from Spark's published sources:
//   PartitionwiseSampledRDD   java.util.Random(seed).nextLong() per partition, in partition order
//   BernoulliSampler(f)       an XORShiftRandom seeded with it; f <= 0.4: GapSamplingIterator
//                             (skip (int)(log(max(u, 5e-11)) / log1p(-f)) rows before the first
//                             and after every kept row), else keep a row when nextDouble() <= f
//   XORShiftRandom.hashSeed   two scala MurmurHash3.bytesHash over ByteBuffer.allocate(Long.SIZE)
//                             (64 bytes: the long big-endian, then zeros)
//   ParallelCollectionRDD     partition p holds rows [p n / N, (p + 1) n / N)
#pragma once

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstring>

namespace eegfx {
namespace spark {

struct JavaRandom {  // java.util.Random (the 48-bit LCG)
  uint64_t s;
  explicit JavaRandom(int64_t seed) : s(((uint64_t)seed ^ 0x5DEECE66DULL) & ((1ULL << 48) - 1)) {}
  int32_t next(int bits) {
    s = (s * 0x5DEECE66DULL + 0xBULL) & ((1ULL << 48) - 1);
    return (int32_t)(uint32_t)(s >> (48 - bits));
  }
  int64_t next_long() {
    const int64_t hi = next(32), lo = next(32);
    return (int64_t)(((uint64_t)hi << 32) + (uint64_t)lo);
  }
};

inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
inline uint32_t mix_last(uint32_t h, uint32_t k) {
  k *= 0xCC9E2D51u;
  k = rotl32(k, 15);
  k *= 0x1B873593u;
  return h ^ k;
}
// scala.util.hashing.MurmurHash3.bytesHash (Scala 2.10) of a length-multiple-of-4 buffer
inline uint32_t murmur3_bytes(const uint8_t* d, int len, uint32_t h) {
  for (int i = 0; i + 4 <= len; i += 4) {
    const uint32_t k = d[i] | (d[i + 1] << 8) | (d[i + 2] << 16) | ((uint32_t)d[i + 3] << 24);
    h = rotl32(mix_last(h, k), 13) * 5u + 0xE6546B64u;
  }
  h ^= (uint32_t)len;
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}

struct XORShiftRandom {  // org.apache.spark.util.random.XORShiftRandom
  uint64_t s;
  explicit XORShiftRandom(int64_t seed) {
    uint8_t buf[64];
    memset(buf, 0, sizeof buf);
    for (int i = 0; i < 8; ++i) buf[i] = (uint8_t)((uint64_t)seed >> (56 - 8 * i));
    const uint32_t lo = murmur3_bytes(buf, 64, 0x3C074A61u);  // MurmurHash3.arraySeed
    const uint32_t hi = murmur3_bytes(buf, 64, lo);
    s = ((uint64_t)hi << 32) | lo;
  }
  int32_t next(int bits) {
    s ^= s << 21;
    s ^= s >> 35;
    s ^= s << 4;
    return (int32_t)(s & ((1ULL << bits) - 1));
  }
  double next_double() {
    return (double)(((int64_t)next(26) << 27) + next(27)) * 0x1.0p-53;
  }
};

// Sets bit r of `mask` (word r / 32) for every row r in [a, b) the partition's sampler keeps
// (the words of [a, b) must be this caller's alone or zero-initialised and written by one thread
// per word); returns the rows kept.
inline int64_t bernoulli_partition(int64_t a, int64_t b, double f, int64_t seed, uint32_t* mask) {
  if (f <= 0.0 || a >= b) return 0;
  int64_t kept = 0;
  auto keep = [&](int64_t r) {
    mask[r >> 5] |= 1u << (r & 31);
    ++kept;
  };
  if (f >= 1.0) {
    for (int64_t r = a; r < b; ++r) keep(r);
    return kept;
  }
  XORShiftRandom rng(seed);
  if (f <= 0.4) {  // RandomSampler.defaultMaxGapSamplingFraction: GapSamplingIterator
    const double lnq = std::log1p(-f);
    auto skip = [&]() -> int64_t {
      const double u = std::max(rng.next_double(), 5e-11);  // RandomSampler.rngEpsilon
      const double k = std::log(u) / lnq;
      return k >= (double)INT_MAX ? (int64_t)INT_MAX : (int64_t)(int32_t)k;  // Double.toInt
    };
    for (int64_t r = a + skip(); r < b; r += 1 + skip()) keep(r);
    return kept;
  }
  for (int64_t r = a; r < b; ++r)
    if (rng.next_double() <= f) keep(r);
  return kept;
}

// RDD.sample(false, f, seed) over n rows in N partitions, as a bit mask (n / 32 words, rounded
// up, cleared here); returns the rows kept.
inline int64_t sample_mask(int64_t n, double f, int32_t N, int64_t seed, uint32_t* mask) {
  memset(mask, 0, sizeof(uint32_t) * (size_t)((n + 31) / 32));
  JavaRandom rnd(seed);
  int64_t kept = 0;
  for (int32_t p = 0; p < N; ++p) {
    const int64_t a = (int64_t)p * n / N, b = (int64_t)(p + 1) * n / N;
    kept += bernoulli_partition(a, b, f, rnd.next_long(), mask);
  }
  return kept;
}

}  // namespace spark
}  // namespace eegfx
