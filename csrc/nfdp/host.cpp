// host.cpp — authoritative flow table (cuckoo), classification-table builders, CPU oracle.
#include "host.h"
#include "shard.h"

#include <cstring>

#include <algorithm>
#include <tuple>

namespace nfdp {

// ------------------------------------------------------------------------------------------
// FlowTableHost
// ------------------------------------------------------------------------------------------
FlowTableHost::FlowTableHost(uint32_t nbuckets_pow2, const std::vector<uint8_t>& rss_key)
    : nb_(nbuckets_pow2), rss_(rss_key) {
  if (nb_ < 2 || (nb_ & (nb_ - 1))) throw std::invalid_argument("nbuckets must be a power of two >= 2");
  if (rss_.size() < 20) throw std::invalid_argument("rss key must be >= 20 bytes");
  slots_.assign((size_t)nb_ * kBucketSlots, FlowSlot{});
}

int FlowTableHost::find_in_bucket(uint32_t b, const FlowKey& k) const {
  const uint32_t used = k.meta | kSlotUsed;
  for (int s = 0; s < kBucketSlots; ++s) {
    const FlowKey& e = slots_[(size_t)b * kBucketSlots + s].key;
    if (e.src_ip == k.src_ip && e.dst_ip == k.dst_ip && e.ports == k.ports && e.meta == used) return s;
  }
  return -1;
}

int64_t FlowTableHost::find(const FlowKey& k) const {
  const TableHash th = table_hash(hash(k), mask());
  int s = find_in_bucket(th.b1, k);
  if (s >= 0) return (int64_t)th.b1 * kBucketSlots + s;
  s = find_in_bucket(th.b2, k);
  if (s >= 0) return (int64_t)th.b2 * kBucketSlots + s;
  return -1;
}

int64_t FlowTableHost::insert(const FlowKey& key, const FlowAction& act) {
  if (key.meta & 0xFF00u & ~kKeyV6) throw std::invalid_argument("FlowKey.meta byte 1 must be zero (but kKeyV6)");
  const int64_t existing = find(key);
  if (existing >= 0) {
    slots_[existing].act = act;
    dirty_.insert((uint32_t)(existing / kBucketSlots));
    return existing;
  }
  FlowKey k = key;
  k.meta |= kSlotUsed;
  FlowAction a = act;
  int64_t first_slot = -1;   // where the NEW key ends up
  int64_t pending_from = -1; // slot the entry currently being placed was evicted from
  uint32_t avoid = 0xFFFFFFFFu;  // bucket the current entry was just evicted from
  // track the path so a failed insert can be rolled back
  std::vector<std::pair<size_t, FlowSlot>> undo;
  std::vector<std::pair<int64_t, int64_t>> new_moves;
  for (int kick = 0; kick < 512; ++kick) {
    FlowKey hk = k;
    hk.meta &= ~kSlotUsed;
    const TableHash cur = table_hash(hash(hk), mask());
    const uint32_t cand[2] = {cur.b1, cur.b2};
    for (int c = 0; c < 2; ++c) {
      for (int s = 0; s < kBucketSlots; ++s) {
        const size_t i = (size_t)cand[c] * kBucketSlots + s;
        if (!(slots_[i].key.meta & kSlotUsed)) {
          slots_[i].key = k; slots_[i].act = a;
          dirty_.insert(cand[c]);
          ++count_;
          if (first_slot < 0) first_slot = (int64_t)i;
          if (pending_from >= 0) new_moves.emplace_back(pending_from, (int64_t)i);
          moves_.insert(moves_.end(), new_moves.begin(), new_moves.end());
          return first_slot;
        }
      }
    }
    // evict a random victim, preferring the bucket the current entry did not come from
    uint32_t vb = cand[rng_() & 1u];
    if (vb == avoid) vb = (vb == cand[0]) ? cand[1] : cand[0];
    const int vs = (int)(rng_() % kBucketSlots);
    const size_t vi = (size_t)vb * kBucketSlots + vs;
    undo.emplace_back(vi, slots_[vi]);
    const FlowKey vk = slots_[vi].key;
    const FlowAction va = slots_[vi].act;
    slots_[vi].key = k; slots_[vi].act = a;
    dirty_.insert(vb);
    if (first_slot < 0) first_slot = (int64_t)vi;
    if (pending_from >= 0) new_moves.emplace_back(pending_from, (int64_t)vi);
    pending_from = (int64_t)vi;
    avoid = vb;
    k = vk; a = va;
  }
  // roll back
  for (auto it = undo.rbegin(); it != undo.rend(); ++it) slots_[it->first] = it->second;
  throw std::runtime_error("flow table full (cuckoo insert failed after 512 kicks)");
}

bool FlowTableHost::erase(const FlowKey& k) {
  const int64_t i = find(k);
  if (i < 0) return false;
  slots_[i] = FlowSlot{};
  dirty_.insert((uint32_t)(i / kBucketSlots));
  --count_;
  return true;
}

std::vector<uint32_t> FlowTableHost::take_dirty() {
  std::vector<uint32_t> v(dirty_.begin(), dirty_.end());
  std::sort(v.begin(), v.end());
  dirty_.clear();
  return v;
}

std::vector<std::pair<int64_t, int64_t>> FlowTableHost::take_moves() {
  auto m = std::move(moves_);
  moves_.clear();
  return m;
}

// ------------------------------------------------------------------------------------------
// ACL (TCAM) tables in the layout of the FP4 MFMA A operand (device.h classify_wave):
// v_mfma_scale_f32_16x16x128_f8f6f4, e2m1: lane l holds rule row (l & 15) of the tile and
// K = 32 (l >> 4) + j for j < 32 as nibble j (little-endian nibbles of 4 dwords); K = key bit,
// LSB-first over the 4 LE key dwords.  Weights: cared bit set -> -1.0 (0xA), cared bit clear ->
// +1.0 (0x2), don't care -> 0; the kernel scales A by 2^12.  C init of the row holding rule r =
// bias_r * 4096 + r (bias = the rule's count of cared set bits), so the accumulator is exactly
// (mismatch << 12) | r and 0 mismatches = a ternary match of rule r.
// Rules are placed in tiles by field signature (similar rules together) and every tile / group
// of kAclGroup tiles gets a prefilter: the key bits all of its rules care about and agree on.
// Output buffer `cinit` = [tiles][4][4] C init | [tiles][8] tile prefilters (mask[4], value[4]) |
// [groups][8] group prefilters.
// ------------------------------------------------------------------------------------------
static inline int key_bit(const uint32_t* w, int b) { return (w[b >> 5] >> (b & 31)) & 1; }
static inline uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

namespace {
// common cared-and-agreeing bits of a rule set -> (mask[4], value[4]); an empty set admits nothing
void prefilter(const uint32_t* value, const uint32_t* mask, const uint32_t* rules, uint32_t nr, uint32_t* out) {
  if (nr == 0) {
    for (int w = 0; w < 4; ++w) { out[w] = 0xFFFFFFFFu; out[4 + w] = 0; }
    out[7] = kSlotUsed;  // key.meta byte 1 is always 0 in a packet key: nothing passes
    return;
  }
  for (int w = 0; w < 4; ++w) {
    uint32_t cm = 0xFFFFFFFFu, diff = 0;
    const uint32_t v0 = value[4 * rules[0] + w] & mask[4 * rules[0] + w];
    for (uint32_t k = 0; k < nr; ++k) {
      const uint32_t r = rules[k];
      cm &= mask[4 * r + w];
      diff |= (value[4 * r + w] & mask[4 * r + w]) ^ v0;
    }
    cm &= ~diff;
    if (w == 3) cm &= ~(kAclSportHi | kAclDportHi);   // prefilters test the flow key: no port-class bits
    out[w] = cm;
    out[4 + w] = v0 & cm;
  }
}
}  // namespace

#ifndef NFDP_ACL_ORDER
#define NFDP_ACL_ORDER 0   // rule placement: 0 protocol, destination, ports, source; 1 source first
#endif
AclFrags build_acl_frags(const uint32_t* value, const uint32_t* mask, uint32_t n) {
  if (n > 4096) throw std::invalid_argument("ACL supports at most 4096 rules (12-bit rule index)");
  AclFrags f;
  f.tiles = (n + 15) / 16;
  if (f.tiles == 0) f.tiles = 1;
  const uint32_t npad = f.tiles * 16;
  const uint32_t groups = (f.tiles + kAclGroupTiles - 1) / kAclGroupTiles;
  // placement: sort by the protocol byte (mask, value) first, then by (dst, ports, src, meta)
  // masks and values in network byte order, so a tile holds rules of one protocol and one shape
  // over neighbouring values (e.g. consecutive /24s, low dports): a group of TCP-only rules then
  // agrees on the protocol byte and its prefilter lets no UDP wave in (and vice versa)
  std::vector<uint32_t> order(n);
  for (uint32_t r = 0; r < n; ++r) order[r] = r;
  auto sig = [&](uint32_t r) {
    const uint32_t* v = value + 4 * r;
    const uint32_t* m = mask + 4 * r;
    auto p16 = [](uint32_t raw) { return ((raw & 0xFFu) << 8) | ((raw >> 8) & 0xFFu); };
    const uint32_t mp = (p16(m[2] >> 16) << 16) | p16(m[2] & 0xFFFFu), vp = (p16(v[2] >> 16) << 16) | p16(v[2] & 0xFFFFu);
    // (then destination: specific prefixes before wildcards, by value, so a group's rules share
    // the destination's leading bits whenever the rule set allows)
#if NFDP_ACL_ORDER == 1
    // source first (then destination, ports): on the ClassBench-style set the tiles' own prefilters
    // admit 29 tiles per wave instead of 37 (tools/acl_prefilter_sim.py --order)
    return std::make_tuple(m[3] & 0xFFu, v[3] & m[3] & 0xFFu, m[0] == 0u, bswap32(v[0] & m[0]), bswap32(m[0]),
                           m[1] == 0u, bswap32(v[1] & m[1]), bswap32(m[1]), mp, vp & mp, m[3], v[3] & m[3], r);
#else
    return std::make_tuple(m[3] & 0xFFu, v[3] & m[3] & 0xFFu, m[1] == 0u, bswap32(v[1] & m[1]), bswap32(m[1]), mp,
                           bswap32(m[0]), m[3], vp & mp, bswap32(v[0] & m[0]), v[3] & m[3], r);
#endif
  };
  std::sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) { return sig(x) < sig(y); });
  f.wfrag.assign((size_t)f.tiles * 64 * 16, 0);
  f.cinit.assign((size_t)f.tiles * 16 + (size_t)f.tiles * 8 + (size_t)groups * 8, 0);
  std::vector<int64_t> row_rule(npad, -1);
  for (uint32_t k = 0; k < n; ++k) row_rule[k] = order[k];
  for (uint32_t nt = 0; nt < f.tiles; ++nt)
    for (int l = 0; l < 64; ++l)
      for (int j = 0; j < 32; ++j) {
        const int64_t r = row_rule[nt * 16 + (l & 15)];
        const int b = 32 * (l >> 4) + j;
        uint8_t w = 0;
        if (r >= 0 && key_bit(mask + 4 * r, b)) w = key_bit(value + 4 * r, b) ? 0xA : 0x2;
        uint8_t& byte = reinterpret_cast<uint8_t&>(f.wfrag[((size_t)nt * 64 + l) * 16 + j / 2]);
        byte = (uint8_t)(byte | (w << (4 * (j & 1))));
      }
  for (uint32_t k = 0; k < npad; ++k) {
    const int64_t r = row_rule[k];
    float c;
    if (r < 0) {
      c = 4096.0f + 4095.0f;  // padding: mismatch >= 1 -> never a match
    } else {
      int32_t bb = 0;
      for (int b = 0; b < 128; ++b)
        if (key_bit(mask + 4 * r, b) && key_bit(value + 4 * r, b)) ++bb;
      c = (float)bb * 4096.0f + (float)r;
    }
    const uint32_t nt = k / 16, row = k % 16;
    std::memcpy(&f.cinit[((size_t)nt * 4 + row / 4) * 4 + row % 4], &c, 4);
  }
  uint32_t* pf = reinterpret_cast<uint32_t*>(f.cinit.data()) + (size_t)f.tiles * 16;
  uint32_t* gpf = pf + (size_t)f.tiles * 8;
  for (uint32_t nt = 0; nt < f.tiles; ++nt) {
    const uint32_t b = nt * 16, e = std::min(n, b + 16);
    prefilter(value, mask, order.data() + b, e > b ? e - b : 0, pf + 8 * nt);
  }
  for (uint32_t g = 0; g < groups; ++g) {
    const uint32_t b = g * 16 * kAclGroupTiles, e = std::min(n, b + 16 * kAclGroupTiles);
    prefilter(value, mask, order.data() + b, e > b ? e - b : 0, gpf + 8 * g);
  }
  // Prefilter tiles: tile t's prefilter (mask, value) as ternary rule row t % 16 of prefilter tile
  // t / 16, in the same FP4 A-fragment / C-init form, so ONE MFMA per 16 packets tests 16 tiles'
  // prefilters at once (device.h classify_wave): accumulator < 4096 <=> no cared bit differs.
  // Appended: wfrag [tiles + ptiles][64][16], cinit ... | [ptiles][4][4] C init.
  const uint32_t ptiles = (f.tiles + 15) / 16;
  f.ptiles = ptiles;
  f.wfrag.resize((size_t)(f.tiles + ptiles) * 64 * 16, 0);
  f.cinit.resize(f.cinit.size() + (size_t)ptiles * 16, 0);
  const uint32_t* pfw = reinterpret_cast<const uint32_t*>(f.cinit.data()) + (size_t)f.tiles * 16;   // (re-read: resized)
  float* pci = reinterpret_cast<float*>(f.cinit.data()) + (size_t)f.tiles * 24 + (size_t)groups * 8;
  for (uint32_t k = 0; k < ptiles * 16; ++k) {
    const uint32_t p = k / 16, row = k % 16;
    float c = 4096.0f + 4095.0f;   // padding row: never passes
    if (k < f.tiles) {
      const uint32_t* m = pfw + 8 * k;
      const uint32_t* v = m + 4;
      int32_t bb = 0;
      for (int b = 0; b < 128; ++b) {
        if (!key_bit(m, b)) continue;
        const int l = 16 * (b / 32) + (int)row, j = b % 32;   // lane (K block, row), nibble j
        const uint8_t w = key_bit(v, b) ? 0xA : 0x2;
        bb += key_bit(v, b);
        uint8_t& byte = reinterpret_cast<uint8_t&>(f.wfrag[(((size_t)f.tiles + p) * 64 + l) * 16 + j / 2]);
        byte = (uint8_t)(byte | (w << (4 * (j & 1))));
      }
      c = (float)bb * 4096.0f + (float)row;
    }
    std::memcpy(&pci[((size_t)p * 4 + row / 4) * 4 + row % 4], &c, 4);
  }
  return f;
}

AclFrags build_acl6_frags(const uint32_t* value, const uint32_t* mask, uint32_t n) {
  if (n > 4096) throw std::invalid_argument("IPv6 ACL supports at most 4096 rules (12-bit rule index)");
  AclFrags f;
  f.tiles = (n + 15) / 16;
  if (f.tiles == 0) f.tiles = 1;
  f.wfrag.assign((size_t)f.tiles * 3 * 64 * 16, 0);
  f.cinit.assign((size_t)f.tiles * 16, 0);
  for (uint32_t nt = 0; nt < f.tiles; ++nt)
    for (int k = 0; k < 3; ++k)
      for (int l = 0; l < 64; ++l)
        for (int j = 0; j < 32; ++j) {
          const uint32_t r = nt * 16 + (l & 15);
          if (r >= n) continue;
          const int b = 32 * (l >> 4) + j;   // bit of words 4k .. 4k+3
          const uint32_t* mw = mask + 12 * (size_t)r + 4 * k;
          const uint32_t* vw = value + 12 * (size_t)r + 4 * k;
          if (!key_bit(mw, b)) continue;
          const uint8_t w = key_bit(vw, b) ? 0xA : 0x2;
          uint8_t& byte = reinterpret_cast<uint8_t&>(f.wfrag[(((size_t)nt * 3 + k) * 64 + l) * 16 + j / 2]);
          byte = (uint8_t)(byte | (w << (4 * (j & 1))));
        }
  for (uint32_t k = 0; k < f.tiles * 16; ++k) {
    float c = 4096.0f + 4095.0f;   // padding row: never a match
    if (k < n) {
      int32_t bb = 0;
      for (int b = 0; b < 384; ++b)
        if (key_bit(mask + 12 * (size_t)k, b) && key_bit(value + 12 * (size_t)k, b)) ++bb;
      c = (float)bb * 4096.0f + (float)k;
    }
    const uint32_t nt = k / 16, row = k % 16;
    std::memcpy(&f.cinit[((size_t)nt * 4 + row / 4) * 4 + row % 4], &c, 4);
  }
  return f;
}

static inline int rss_bit(const uint8_t* key, int x) { return (key[x >> 3] >> (7 - (x & 7))) & 1; }

std::vector<int8_t> build_toeplitz_frags(const uint8_t* rss_key) {
  std::vector<int8_t> f(2 * 2 * 64 * 16, 0);
  for (int m = 0; m < 2; ++m)
    for (int s = 0; s < 2; ++s)
      for (int l = 0; l < 64; ++l)
        for (int j = 0; j < 16; ++j) {
          const int ncol = 16 * m + (l & 15);              // window offset
          const int b = 64 * s + 16 * (l >> 4) + j;        // key bit (LSB-first LE)
          const int i = 8 * (b >> 3) + (7 - (b & 7));      // Toeplitz input bit (MSB-first)
          f[(((size_t)m * 2 + s) * 64 + l) * 16 + j] = (int8_t)rss_bit(rss_key, i + ncol);
        }
  return f;
}

std::vector<uint32_t> build_toeplitz_table(const uint8_t* rss_key) {
  std::vector<uint32_t> t(16 * 256, 0);
  for (int pos = 0; pos < 16; ++pos)
    for (int v = 0; v < 256; ++v) {
      uint32_t h = 0;
      for (int bit = 7; bit >= 0; --bit) {
        if (!(v & (1 << bit))) continue;
        const int i = 8 * pos + (7 - bit);
        uint32_t win = 0;
        for (int q = 0; q < 32; ++q) win = (win << 1) | (uint32_t)rss_bit(rss_key, i + q);
        h ^= win;
      }
      t[pos * 256 + v] = h;
    }
  return t;
}

// ------------------------------------------------------------------------------------------
// CPU oracle
// ------------------------------------------------------------------------------------------
namespace {
// Sequential sink of pipeline.h side_stage (replica positions in packet order; the GPU's are in
// atomic order, so tests compare replica sets).
struct CpuSideSink {
  const SideOut& so;
  uint64_t* port_ctr;
  uint64_t* drop_ctr;
  void rep(const uint32_t* hdr, uint32_t meta, uint32_t src) {
    const uint32_t pos = so.cnt[0]++;
    if (pos >= so.cap_rep) { ++so.cnt[2]; return; }
    std::memcpy(so.rep_hdr + (size_t)pos * kSlotDwords, hdr, kSlotBytes);
    so.rep_meta[pos] = meta;
    so.rep_src[pos] = src;
    const uint32_t r = meta_reason(meta), port = meta_port(meta);
    if (r) { if (drop_ctr) drop_ctr[r] += 1; }
    else if (port < (uint32_t)kMaxPorts && port_ctr) port_ctr[2 * port + 1] += ctr_inc(meta_len(meta));
  }
  void xhdr(const uint32_t* hdr, uint32_t src, uint32_t) {   // (the whole record: zero tail included)
    if (so.xhdr) std::memcpy(so.xhdr + (size_t)src * (kXhdrBytes / 4), hdr, kXhdrBytes);
  }
  void learn(uint32_t bridge, uint32_t lo, uint32_t hi, uint32_t port) {
    const uint32_t pos = so.cnt[1]++;
    if (pos >= so.cap_learn) { ++so.cnt[3]; return; }
    uint32_t* e = so.learn + (size_t)pos * 4;
    e[0] = lo; e[1] = (hi & 0xFFFFu) | (bridge << 16); e[2] = port; e[3] = 0;
  }
};
}  // namespace

uint32_t mac_learn_cpu(MacEntry* macs, uint32_t mask, const uint32_t* ev, uint32_t n, uint32_t stamp) {
  uint32_t dropped = 0;
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t lo = ev[4 * i], hi = ev[4 * i + 1] & 0xFFFFu, br = ev[4 * i + 1] >> 16, port = ev[4 * i + 2];
    const uint32_t h = mac_hash(br, lo, hi) & mask;
    bool done = false;
    for (int probe = 0; probe < 16 && !done; ++probe) {
      MacEntry& e = macs[(h + probe) & mask];
      if (e.valid == kMacEmpty) {
        e.mac_lo = lo; e.mac_hi = (uint16_t)hi; e.bridge_id = (uint16_t)br; e.out_port = (uint16_t)port;
        e.valid = kMacLearned; e.stamp = stamp;
        done = true;
      } else if ((e.valid == kMacStatic || e.valid == kMacLearned) && e.mac_lo == lo && e.mac_hi == hi &&
                 e.bridge_id == br) {
        if (e.valid == kMacLearned) { e.out_port = (uint16_t)port; e.stamp = stamp; }
        done = true;
      }
    }
    if (!done) ++dropped;
  }
  return dropped;
}

void oracle_run(const TablesView& t, const uint32_t* pkts, const uint32_t* inmeta, uint32_t n,
                uint32_t* out, uint32_t* out_meta, uint64_t* flow_ctr, uint64_t* port_ctr,
                uint64_t* drop_ctr, uint32_t* hashes, int32_t* acl_rules, const SideOut* side,
                HopState* hop_state) {
  uint32_t prev_ci = (uint32_t)kSlotBytes << 8;   // strip | hv << 8 of the previous slot when it heads a pair
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t* d = pkts + (size_t)i * kSlotDwords;
    // wide header pairs (pipeline.h decap_pair): a continuation belongs to the slot before it
    uint32_t im = inmeta[i], ci = (uint32_t)kSlotBytes << 8;
    uint32_t inner[kSlotDwords];
    const bool cont = (im & 0xFFFFu) == kPortCont;
    if (!cont && i + 1 < n && (inmeta[i + 1] & 0xFFFFu) == kPortCont) {
      uint32_t strip, hv;
      const int tp = decap_pair(t, DirectTables{t}, d, pkts + (size_t)(i + 1) * kSlotDwords, im, inner, strip, hv);
      if (tp >= 0) {
        if (port_ctr) port_ctr[2 * (im & 0xFFFFu)] += ctr_inc(im >> 16);   // the outer frame on its VTEP port
        d = inner;
        im = (uint32_t)tp | (((im >> 16) - strip) << 16);
        ci = strip | (hv << 8);
      }
    }
    Parsed p;
    IngressState st;
    ingress_stage(t, d, im, p, st);
    if (cont) { st.reason = kCont; st.in_ext = i ? prev_ci : ((uint32_t)kSlotBytes << 8); }
    prev_ci = ci;
    const uint32_t h = toeplitz_scalar(st.key, t.rss_key);
    const int acl = acl_rule_scalar(t, p, st);
    if (hashes) hashes[i] = h;
    if (acl_rules) acl_rules[i] = acl;
    bool hit = false;
    FlowAction act = {};
    if (!st.reason && flowable(t, p)) {
      int64_t slot = flow_lookup(t, st.key, h);
      if (slot >= 0 && p.ipv6 && !flow6_verify(t, p, slot)) slot = -1;
      if (slot >= 0) {
        hit = true;
        act = t.flows[slot].act;
        if (flow_ctr) flow_ctr[slot] += ctr_inc(st.wire_len);
      }
    }
    const EgressDecision e = chain_stage(t, p, st, hit, act, acl, h);
    uint32_t o[kSlotDwords];
    emit(p, e.tci, e.push != 0, o);
    const uint32_t olen = out_len(p, e);
    std::memcpy(out + (size_t)i * kSlotDwords, o, sizeof(o));
    out_meta[i] = make_meta(e.out_port, olen, e.reason, !e.reason && e.xhdr, !e.reason && e.flood);
    if (hop_state && e.reason == kRemote && e.inner_len) hop_state[i] = hop_state_of(p, st, e, act, acl, h);
    if (side && side->cnt && side_needed(st, p, e)) {
      const uint32_t q = side->cnt[5]++;
      if (q < side->cap_list) side->list[q] = i;
      else ++side->cnt[6];
    }
    if (port_ctr) {
      if (st.in_port < (uint32_t)kMaxPorts) port_ctr[2 * st.in_port] += ctr_inc(st.wire_len);
      if (!e.reason) port_ctr[2 * e.out_port + 1] += ctr_inc(olen);
    }
    if (drop_ctr && e.reason) drop_ctr[e.reason & (kNumReasons - 1)] += 1;
  }
  // side pass (GPU: side_kernel after the fused kernel); a terminated pair head works on its inner frame
  if (side && side->cnt) {
    CpuSideSink sk{*side, port_ctr, drop_ctr};
    const uint32_t nl = std::min(side->cnt[5], side->cap_list);
    for (uint32_t j = 0; j < nl; ++j) {
      const uint32_t i = side->list[j];
      const uint32_t* d = pkts + (size_t)i * kSlotDwords;
      uint32_t im = inmeta[i], inner[kSlotDwords];
      if (i + 1 < n && (im & 0xFFFFu) != kPortCont && (inmeta[i + 1] & 0xFFFFu) == kPortCont) {
        uint32_t strip, hv;
        const int tp = decap_pair(t, DirectTables{t}, d, pkts + (size_t)(i + 1) * kSlotDwords, im, inner, strip, hv);
        if (tp >= 0) { d = inner; im = (uint32_t)tp | (((im >> 16) - strip) << 16); }
      }
      side_stage(t, DirectTables{t}, d, im, out + (size_t)i * kSlotDwords, out_meta[i], i, sk);
    }
  }
}

void oracle_resume(const TablesView& t, const uint32_t* hdr, const HopState* state, uint32_t n, uint32_t* out,
                   uint32_t* out_meta, HopState* out_state, uint64_t* port_ctr, uint64_t* drop_ctr) {
  const DirectTables ta{t};
  for (uint32_t i = 0; i < n; ++i) {
    const HopState hs = state[i];
    Parsed p;
    IngressState st;
    resume_ingress(ta, hdr + (size_t)i * kSlotDwords, hs.inmeta, p, st);
    const EgressDecision e = resume_stage(t, ta, p, st, hs.act, hs.acl_rule, hs.hash, hs.hop);
    uint32_t o[kSlotDwords];
    emit(p, e.tci, e.push != 0, o);
    const uint32_t olen = out_len(p, e);
    std::memcpy(out + (size_t)i * kSlotDwords, o, sizeof(o));
    out_meta[i] = make_meta(e.out_port, olen, e.reason, !e.reason && e.xhdr, false);
    if (out_state && e.reason == kRemote && e.inner_len) out_state[i] = hop_state_of(p, st, e, hs.act, hs.acl_rule, hs.hash);
    if (port_ctr && !e.reason) port_ctr[2 * e.out_port + 1] += ctr_inc(olen);
    if (drop_ctr && e.reason) drop_ctr[e.reason & (kNumReasons - 1)] += 1;
  }
}

void oracle_run_remote(const TablesView& t, const uint32_t* pkts, const uint32_t* inmeta, uint32_t n,
                       uint32_t* out, uint32_t* out_meta, uint64_t* flow_ctr, uint64_t* port_ctr,
                       uint64_t* drop_ctr, const RemoteOut& r) {
  const size_t pseg = pkt_seg_bytes(r.cap_pkt);
  uint32_t prev_ci = (uint32_t)kSlotBytes << 8;   // strip | hv << 8 of the previous slot when it heads a pair
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t* d = pkts + (size_t)i * kSlotDwords;
    // wide header pairs (pipeline.h decap_pair): a continuation belongs to the slot before it
    uint32_t im = inmeta[i], ci = (uint32_t)kSlotBytes << 8;
    uint32_t inner[kSlotDwords];
    const bool cont = (im & 0xFFFFu) == kPortCont;
    if (!cont && i + 1 < n && (inmeta[i + 1] & 0xFFFFu) == kPortCont) {
      uint32_t strip, hv;
      const int tp = decap_pair(t, DirectTables{t}, d, pkts + (size_t)(i + 1) * kSlotDwords, im, inner, strip, hv);
      if (tp >= 0) {
        if (port_ctr) port_ctr[2 * (im & 0xFFFFu)] += ctr_inc(im >> 16);   // the outer frame on its VTEP port
        d = inner;
        im = (uint32_t)tp | (((im >> 16) - strip) << 16);
        ci = strip | (hv << 8);
      }
    }
    Parsed p;
    IngressState st;
    ingress_stage(t, d, im, p, st);
    if (cont) { st.reason = kCont; st.in_ext = i ? prev_ci : ((uint32_t)kSlotBytes << 8); }
    prev_ci = ci;
    const uint32_t h = toeplitz_scalar(st.key, t.rss_key);
    const int acl = acl_rule_scalar(t, p, st);
    // flow-owner steering: another GPU's flow goes to its owner as it came in
    const uint32_t owner = owner_of(h, r.nranks);
    const bool to_owner = r.steer && !st.reason && flowable(t, p) && owner != r.rank && im == inmeta[i];   // (terminated: stays)
    if (to_owner) st.reason = kRemote;
    bool hit = false;
    FlowAction act = {};
    if (!st.reason && flowable(t, p)) {
      int64_t slot = flow_lookup(t, st.key, h);
      if (slot >= 0 && p.ipv6 && !flow6_verify(t, p, slot)) slot = -1;
      if (slot >= 0) {
        hit = true;
        act = t.flows[slot].act;
        if (flow_ctr) flow_ctr[slot] += ctr_inc(st.wire_len);
      }
    }
    const EgressDecision e = chain_stage(t, p, st, hit, act, acl, h);
    const uint32_t eg = r.steer ? owner : (e.reason ? r.rank : (uint32_t)t.ports[e.out_port].gpu);
    const bool remote = r.steer ? to_owner : (!e.reason && eg != r.rank && eg < r.nranks);
    uint32_t reason = e.reason;
    uint32_t pos = 0;
    if (remote) {
      pos = r.pcnt[eg]++;
      if (pos >= r.cap_pkt) reason = kOverflow;
    }
    uint32_t o[kSlotDwords];
    emit(p, to_owner ? p.tci : e.tci, to_owner ? p.tagged : e.push != 0, o);
    const uint32_t olen = reason == e.reason ? egress_len(p, e) : 0u;
    const bool to_peer = remote && reason != kOverflow;
    if (to_peer) {
      uint8_t* segp = r.send_pkt + eg * pseg;
      std::memcpy(segp + 64 + (size_t)pos * 64, o, sizeof(o));
      const uint32_t m = r.steer ? inmeta[i] : make_meta(e.out_port, olen, kOk, e.xhdr != 0);
      std::memcpy(segp + pkt_meta_off(r.cap_pkt) + 4 * (size_t)pos, &m, 4);
      out_meta[i] = make_meta(r.steer ? kPortNone : e.out_port, r.steer ? st.wire_len : olen, kRemote);
    } else {
      std::memcpy(out + (size_t)i * kSlotDwords, o, sizeof(o));
      out_meta[i] = make_meta(reason == kOverflow ? kPortNone : e.out_port, olen, reason, !reason && e.xhdr,
                              !reason && e.flood);
    }
    const bool counted_by_owner = to_owner && to_peer;
    if (port_ctr && !counted_by_owner) {
      if (st.in_port < (uint32_t)kMaxPorts) port_ctr[2 * st.in_port] += ctr_inc(st.wire_len);
      if (!reason && !to_peer) port_ctr[2 * e.out_port + 1] += ctr_inc(olen);
    }
    if (drop_ctr && reason && !counted_by_owner) drop_ctr[reason & (kNumReasons - 1)] += 1;
  }
  for (uint32_t o = 0; o < r.nranks; ++o) {
    const uint32_t hdr[4] = {r.pcnt[o] < r.cap_pkt ? r.pcnt[o] : r.cap_pkt, r.cap_pkt, 0, 0};
    std::memcpy(r.send_pkt + o * pseg, hdr, 16);
  }
}

uint32_t gather_cpu(const uint8_t* recv, uint32_t nranks, uint32_t rank, uint32_t cap, uint32_t seg_bytes,
                    uint32_t meta_off, uint32_t* pkts, uint32_t* inmeta) {
  uint32_t n = 0;
  for (uint32_t s = 0; s < nranks; ++s) {
    if (s == rank) continue;
    const uint8_t* seg = recv + (size_t)s * seg_bytes;
    uint32_t c;
    std::memcpy(&c, seg, 4);
    c = std::min(c, cap);
    std::memcpy(pkts + (size_t)n * kSlotDwords, seg + 64, (size_t)c * kSlotBytes);
    std::memcpy(inmeta + n, seg + meta_off, (size_t)c * 4);
    n += c;
  }
  return n;
}

}  // namespace nfdp
