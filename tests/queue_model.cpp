// CPU stress model of the fused frame's queue protocol (vrt_render.hip, frame_kernel + drain_kernel).
// Threads play the waves of one launch: heavy-pass waves of class r append to segment A_r, the
// others to B_s; a wave appends 1..31 exact pixels (or renders >= 32 in place: no append). Batches
// are fixed index ranges [B k, B (k + 1)) of a segment, owned by the wave whose reservation covers
// the batch's last index; the heavy-pass wave that completes class r (a per-class counter) owns the
// partial last batch of A_r; after every thread has joined, the "drain kernel" owns the partial last
// batches of the B segments. Checks: every queued pixel rendered exactly once, no batch read past
// the reservations, every entry wait satisfied. Test infrastructure only (tests/test_queue_protocol.py).
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <random>
#include <thread>
#include <vector>

constexpr uint32_t kClasses = 8, B = 64, kEpoch = 7;
struct Seg {
  std::atomic<uint32_t> tail{0};
  std::vector<std::atomic<uint64_t>> ent;
};
Seg segA[kClasses], segB[kClasses];
std::atomic<uint32_t> hcls[kClasses];
std::vector<std::atomic<int>> seen;
std::atomic<long> bad{0};
uint32_t cls_waves[kClasses];

uint32_t entry(Seg& s, uint32_t i) {
  if (i >= s.ent.size()) { bad++; return ~0u; }
  uint64_t v;
  long spins = 0;
  while (((v = s.ent[i].load()) >> 32) != kEpoch) {
    if (++spins > 100000000) { bad++; return ~0u; }
    std::this_thread::yield();
  }
  return uint32_t(v);
}
void render(uint32_t id) { if (id != ~0u) seen[id].fetch_add(1); }

void wave(int id, uint32_t cnt, bool heavy, uint32_t cls) {
  std::mt19937 rng(id);
  Seg& s = heavy ? segA[cls] : segB[cls];
  uint32_t kb0 = 0, kb1 = 0;
  if (cnt && cnt < 32) {
    const uint32_t base = s.tail.fetch_add(cnt);
    for (uint32_t r = 0; r < cnt; ++r) {
      if (rng() % 4 == 0) std::this_thread::yield();
      if (base + r < s.ent.size()) s.ent[base + r].store((uint64_t(kEpoch) << 32) | (id * 64 + r));
    }
    kb0 = base / B;            // frame_kernel: (base + B) / B - 1
    kb1 = (base + cnt) / B;
  } else if (cnt >= 32) {
    for (uint32_t r = 0; r < cnt; ++r) render(id * 64 + r);   // in place
  }
  uint32_t lo = 0, hi = 0;
  if (heavy && hcls[cls].fetch_add(1) + 1 == cls_waves[cls]) {
    const uint32_t t = segA[cls].tail.load();
    lo = t / B * B;
    hi = t;
  }
  for (uint32_t k = kb0; k < kb1; ++k)
    for (uint32_t l = 0; l < B; ++l) render(entry(s, k * B + l));
  for (uint32_t i = lo; i < hi; ++i) render(entry(segA[cls], i));
}

int main() {
  for (int trial = 0; trial < 200; ++trial) {
    std::mt19937 rng(trial);
    const int waves = 200 + rng() % 300;
    const bool heavy_pass = trial % 3 != 0;
    seen = std::vector<std::atomic<int>>(size_t(waves) * 64);
    std::vector<uint32_t> cnt(waves), cls(waves);
    std::vector<bool> hv(waves);
    for (uint32_t r = 0; r < kClasses; ++r) {
      cls_waves[r] = 0;
      hcls[r] = 0;
    }
    for (int i = 0; i < waves; ++i) {
      const uint32_t x = rng() % 10;
      cnt[i] = x < 5 ? 0 : (x < 9 ? rng() % 31 + 1 : 32 + rng() % 33);
      hv[i] = heavy_pass && i < waves / 4;
      cls[i] = i % kClasses;
      if (hv[i]) cls_waves[cls[i]]++;
    }
    for (uint32_t r = 0; r < kClasses; ++r) {
      segA[r].tail = 0;
      segB[r].tail = 0;
      segA[r].ent = std::vector<std::atomic<uint64_t>>(size_t(waves) * 31);
      segB[r].ent = std::vector<std::atomic<uint64_t>>(size_t(waves) * 31);
      for (auto& e : segA[r].ent) e.store(0);
      for (auto& e : segB[r].ent) e.store(0);
    }
    std::vector<std::thread> th;
    for (int i = 0; i < waves; ++i) th.emplace_back(wave, i, cnt[i], bool(hv[i]), cls[i]);
    for (auto& t : th) t.join();
    // drain kernel: the partial last batches of the B segments
    for (uint32_t r = 0; r < kClasses; ++r) {
      const uint32_t t = segB[r].tail.load();
      for (uint32_t i = t / B * B; i < t; ++i) render(entry(segB[r], i));
    }
    for (int i = 0; i < waves; ++i)
      for (uint32_t r = 0; r < 64; ++r) {
        const int want = r < cnt[i] ? 1 : 0;
        if (seen[size_t(i) * 64 + r] != want) {
          printf("trial %d wave %d pixel %u rendered %d times\n", trial, i, r, int(seen[size_t(i) * 64 + r]));
          return 1;
        }
      }
    if (bad) {
      printf("trial %d: %ld bad reads\n", trial, long(bad));
      return 1;
    }
  }
  printf("ok\n");
  return 0;
}
