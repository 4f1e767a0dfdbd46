// CPU stress model of frame_kernel's queue protocol (vrt_render.hip, "fused frame"): threads play
// waves that append 0..31 exact pixels (or >= 32: in place, no append), publish done / hdone, and
// then claim batches (full batches at any time, partial ones once the heavy pass or every wave is
// done: the flags their last waves set) exactly as queue_claim does, reading flags, head, tail in
// that order; only waves that appended, set a flag or rendered a batch poll (as frame_kernel). Checks that every
// queued pixel is rendered exactly once and no claim reaches past the reservations. Test
// infrastructure only (tests/test_queue_protocol.py); the order of the head and tail reads is the
// one a reversed version gets wrong (claims past the tail, waits for entries never written).
#include <atomic>
#include <cstdio>
#include <cstdint>
#include <random>
#include <thread>
#include <vector>
std::atomic<uint32_t> tail{0}, head{0}, done_{0}, hdone{0}, flags{0};
std::vector<std::atomic<uint64_t>> ent;
std::vector<std::atomic<int>> seen;
uint32_t total, heavy_total, cap; const uint32_t B = 64, epoch = 7;
std::atomic<long> bad{0};
void wave(int id, uint32_t cnt, bool heavy, bool inplace) {
  std::mt19937 rng(id);
  const bool appended = cnt && !inplace;
  if (appended) {
    uint32_t base = tail.fetch_add(cnt);
    for (uint32_t r = 0; r < cnt; ++r) {
      if (rng() % 4 == 0) std::this_thread::yield();
      if (base + r < cap) ent[base + r].store((uint64_t(epoch) << 32) | (id * 64 + r));
    }
  }
  // completion: the last wave sets flag 2, the heavy pass's last wave flag 1 (kernel: sharded
  // counters whose last adder counts the shard; one counter here)
  uint32_t fl = 0;
  if (done_.fetch_add(1) + 1 == total) fl |= 2;
  if (heavy && hdone.fetch_add(1) + 1 == heavy_total) fl |= 1;
  if (fl) flags.fetch_or(fl);
  // poll only when something this wave did can have made a batch claimable
  bool poll = appended || fl || inplace;
  for (;;) {
    if (!poll) break;
    uint32_t h = 0, want = 0;
    for (int tries = 0; tries < (1 << 20); ++tries) {
      uint32_t f = flags.load();
      h = head.load();
      if (rng() % 8 == 0) std::this_thread::yield();
      uint32_t t = tail.load();
      uint32_t avail = t > h ? t - h : 0;
      uint32_t w = avail >= B ? B : 0;
      if (avail && !w && (heavy_total == 0 || f)) w = avail;
      if (!w) break;
      uint32_t e = h;
      if (head.compare_exchange_strong(e, h + w)) { want = w; break; }
    }
    if (!want) break;
    for (uint32_t l = 0; l < want; ++l) {
      if (h + l >= cap) { bad++; continue; }
      uint64_t v; long spins = 0;
      while (((v = ent[h + l].load()) >> 32) != epoch) { if (++spins > 100000000) { bad++; break; } std::this_thread::yield(); }
      seen[uint32_t(v)].fetch_add(1);
    }
    poll = true;
  }
}
int main() {
  for (int trial = 0; trial < 200; ++trial) {
    std::mt19937 rng(trial);
    int waves = 200 + rng() % 200; total = waves; cap = waves * 31;
    ent = std::vector<std::atomic<uint64_t>>(cap); seen = std::vector<std::atomic<int>>(waves * 64);
    for (auto& e : ent) e.store(0);
    tail = head = done_ = hdone = flags = 0;
    std::vector<uint32_t> cnt(waves); std::vector<bool> hv(waves);
    uint32_t nheavy = 0; long expected = 0;
    for (int i = 0; i < waves; ++i) {
      uint32_t r = rng() % 10; cnt[i] = r < 6 ? 0 : (r < 9 ? rng() % 31 + 1 : 32 + rng() % 33);
      hv[i] = i < waves / 5; nheavy += hv[i];
      if (cnt[i] && cnt[i] < 32) expected += cnt[i];
    }
    heavy_total = (trial % 3 == 0) ? 0 : nheavy;
    std::vector<std::thread> th;
    for (int i = 0; i < waves; ++i) th.emplace_back(wave, i, cnt[i], hv[i], cnt[i] >= 32);
    for (auto& t : th) t.join();
    long got = 0, dup = 0;
    for (int i = 0; i < waves; ++i) for (uint32_t r = 0; r < 64; ++r) { int s = seen[i * 64 + r]; got += s; if (s > 1) dup++; if (cnt[i] && cnt[i] < 32 && r < cnt[i] && s != 1) { printf("trial %d wave %d entry %u seen %d\n", trial, i, r, s); return 1; } }
    if (got != expected || dup || bad) { printf("trial %d: got %ld expected %ld dup %ld bad %ld\n", trial, got, expected, dup, long(bad)); return 1; }
  }
  printf("ok\n");
}
