// IPsec ESP (RFC 4303) with AES-GCM (RFC 4106, 16-B ICV, 8-B explicit IV) on the data plane:
// the MI355X take on the IPU's inline crypto engine behind the P4 pipeline's IPsec tables
// (ipsec_spd, ipsec_tx_sa_classification_table, ipsec_tunnel_encap_mod_table,
// ipsec_rx_sa_classification_table, ipv4_ipsec_tunnel_term_table:
// fxp-net_linux-networking.p4info.txt).  Crypto runs on whole frames at the port boundary, before
// (inbound) or after (outbound) the header pipeline.
//
// One lane per packet.  Frames are staged with a headroom chosen so every plaintext and
// ciphertext dword is 4-B aligned: cleartext frames at slot + 2 (the IP header at slot + 16, as
// NET_IP_ALIGN does), ESP frames at slot + 14 (50 header bytes, ciphertext at slot + 64).
// AES uses the big-endian-word T-table formulation (Te0 + rotations, S-box for the last round);
// GHASH uses 4-bit tables of H per SA (Shoup's method).  Everything here is __host__ __device__:
// the oracle (ipsec_cpu.cpp) runs the same per-packet functions.
#pragma once
#include "nfdp.h"

namespace nfdp {

constexpr uint32_t kEspTunnel = 1, kEspTransport = 2;
constexpr int kClearOff = 2;   // cleartext frame offset in its slot
constexpr int kEspOff = 14;    // ESP frame offset in its slot
constexpr int kEspHdrBytes = 50;   // Ethernet 14 + IPv4 20 + SPI/seq 8 + IV 8
constexpr int kEspIcv = 16;
constexpr int kEspMaxSa = 4096;

// status codes (per packet)
enum EspStatus : uint32_t {
  kEspBypass = 0,     // outbound: SPD bypass / no entry (the frame leaves as it is)
  kEspDone = 1,       // encrypted / decrypted and authenticated
  kEspDrop = 2,       // SPD drop, malformed frame or no room in the output slot
  kEspAuthFail = 3,   // inbound: ICV mismatch or bad trailer
  kEspNoSa = 4,       // inbound: no SA for (src, dst, SPI): slow path
};

struct alignas(16) EspSa {       // 4384 B
  uint32_t rk[60];               // AES round keys, big-endian words; 4 * (nr + 1) used
  uint32_t nr;                   // 10 (AES-128-GCM) / 14 (AES-256-GCM); 0 = empty slot
  uint32_t salt;                 // RFC 4106 salt: the 4 key-material bytes, raw (network order)
  uint32_t spi;                  // host order
  uint32_t mode;                 // kEspTunnel / kEspTransport
  uint32_t src_ip, dst_ip;       // tunnel mode outer addresses, raw
  uint32_t smac_lo, dmac_lo;     // tunnel mode outer MACs (raw bytes 0..3)
  uint16_t smac_hi, dmac_hi;
  uint32_t pad[3];
  uint64_t htab[256][2];         // GHASH 8-bit table: byte b (as the block's first byte) times
                                 // H = E_K(0), (hi, lo) 64-bit halves of the big-endian block
};
static_assert(sizeof(EspSa) == 4384, "EspSa");

// ipsec_spd + ipsec_tx_sa_classification: (dst IPv4, protocol) -> protect with SA / bypass / drop
enum SpdAction : uint8_t { kSpdEmpty = 0, kSpdProtect = 1, kSpdBypass = 2, kSpdDrop = 3 };
struct alignas(16) SpdEntry {
  uint32_t dst_ip;               // raw
  uint8_t proto, action;
  uint16_t sa;
  uint32_t pad[2];
};
static_assert(sizeof(SpdEntry) == 16, "SpdEntry");
// ipsec_rx_sa_classification_table: (outer src, outer dst, SPI) -> SA
struct alignas(16) RxSaEntry {
  uint32_t src_ip, dst_ip;       // raw
  uint32_t spi;                  // host order
  uint16_t sa, valid;
};
static_assert(sizeof(RxSaEntry) == 16, "RxSaEntry");

NFDP_HD uint32_t spd_hash(uint32_t dst, uint32_t proto) { return fmix32(dst ^ (proto * 0x9E3779B1u)); }
NFDP_HD uint32_t rxsa_hash(uint32_t src, uint32_t dst, uint32_t spi) {
  return fmix32(src ^ (dst * 0x85EBCA6Bu) ^ (spi * 0xC2B2AE35u));
}

NFDP_HD uint32_t bswap32_(uint32_t x) {
  return (x >> 24) | ((x >> 8) & 0xFF00u) | ((x << 8) & 0xFF0000u) | (x << 24);
}
NFDP_HD uint32_t rotr32(uint32_t x, int r) { return (x >> r) | (x << (32 - r)); }

#ifndef NFDP_ESP_TTABLES4
#define NFDP_ESP_TTABLES4 1   // four T-tables (4 KB of LDS) instead of Te0 + rotations
#endif

// Table access (LDS on the GPU, plain arrays on the host).
struct EspTables {
  const uint32_t* te0;   // [256] (2s, s, s, 3s) big-endian word of S-box byte s; with
                         // NFDP_ESP_TTABLES4 [4][256]: Te0 and its byte rotations Te1..Te3
  const uint8_t* sbox;   // [256]
  const uint64_t* rem;   // [256] GHASH 8-bit reduction constants
};

// AES encryption of one block given as 4 big-endian words.
NFDP_HD void aes_block(const EspTables& tb, const uint32_t* rk, uint32_t nr, const uint32_t in[4], uint32_t out[4]) {
  uint32_t s0 = in[0] ^ rk[0], s1 = in[1] ^ rk[1], s2 = in[2] ^ rk[2], s3 = in[3] ^ rk[3];
  const uint32_t* te = tb.te0;
  for (uint32_t r = 1; r < nr; ++r) {
    const uint32_t* k = rk + 4 * r;
#if NFDP_ESP_TTABLES4
    const uint32_t *e1 = te + 256, *e2 = te + 512, *e3 = te + 768;
    const uint32_t t0 = te[s0 >> 24] ^ e1[(s1 >> 16) & 0xFF] ^ e2[(s2 >> 8) & 0xFF] ^ e3[s3 & 0xFF] ^ k[0];
    const uint32_t t1 = te[s1 >> 24] ^ e1[(s2 >> 16) & 0xFF] ^ e2[(s3 >> 8) & 0xFF] ^ e3[s0 & 0xFF] ^ k[1];
    const uint32_t t2 = te[s2 >> 24] ^ e1[(s3 >> 16) & 0xFF] ^ e2[(s0 >> 8) & 0xFF] ^ e3[s1 & 0xFF] ^ k[2];
    const uint32_t t3 = te[s3 >> 24] ^ e1[(s0 >> 16) & 0xFF] ^ e2[(s1 >> 8) & 0xFF] ^ e3[s2 & 0xFF] ^ k[3];
#else
    const uint32_t t0 = te[s0 >> 24] ^ rotr32(te[(s1 >> 16) & 0xFF], 8) ^ rotr32(te[(s2 >> 8) & 0xFF], 16) ^
                        rotr32(te[s3 & 0xFF], 24) ^ k[0];
    const uint32_t t1 = te[s1 >> 24] ^ rotr32(te[(s2 >> 16) & 0xFF], 8) ^ rotr32(te[(s3 >> 8) & 0xFF], 16) ^
                        rotr32(te[s0 & 0xFF], 24) ^ k[1];
    const uint32_t t2 = te[s2 >> 24] ^ rotr32(te[(s3 >> 16) & 0xFF], 8) ^ rotr32(te[(s0 >> 8) & 0xFF], 16) ^
                        rotr32(te[s1 & 0xFF], 24) ^ k[2];
    const uint32_t t3 = te[s3 >> 24] ^ rotr32(te[(s0 >> 16) & 0xFF], 8) ^ rotr32(te[(s1 >> 8) & 0xFF], 16) ^
                        rotr32(te[s2 & 0xFF], 24) ^ k[3];
#endif
    s0 = t0; s1 = t1; s2 = t2; s3 = t3;
  }
  const uint8_t* sb = tb.sbox;
  const uint32_t* k = rk + 4 * nr;
  out[0] = (((uint32_t)sb[s0 >> 24] << 24) | ((uint32_t)sb[(s1 >> 16) & 0xFF] << 16) |
            ((uint32_t)sb[(s2 >> 8) & 0xFF] << 8) | sb[s3 & 0xFF]) ^ k[0];
  out[1] = (((uint32_t)sb[s1 >> 24] << 24) | ((uint32_t)sb[(s2 >> 16) & 0xFF] << 16) |
            ((uint32_t)sb[(s3 >> 8) & 0xFF] << 8) | sb[s0 & 0xFF]) ^ k[1];
  out[2] = (((uint32_t)sb[s2 >> 24] << 24) | ((uint32_t)sb[(s3 >> 16) & 0xFF] << 16) |
            ((uint32_t)sb[(s0 >> 8) & 0xFF] << 8) | sb[s1 & 0xFF]) ^ k[2];
  out[3] = (((uint32_t)sb[s3 >> 24] << 24) | ((uint32_t)sb[(s0 >> 16) & 0xFF] << 16) |
            ((uint32_t)sb[(s1 >> 8) & 0xFF] << 8) | sb[s2 & 0xFF]) ^ k[3];
}

// X = X * H in GF(2^128) (GCM bit order), X as (hi, lo) of the big-endian block; 8-bit table
// (Shoup): one table entry and one reduction constant per byte, last byte first.
NFDP_HD void ghash_mul(const EspTables& tb, const uint64_t (*ht)[2], uint64_t& xh, uint64_t& xl) {
  uint64_t zh = 0, zl = 0;
#pragma unroll
  for (int cnt = 15; cnt >= 0; --cnt) {
    const uint32_t b = cnt >= 8 ? (uint32_t)(xl >> (8 * (15 - cnt))) & 0xFFu : (uint32_t)(xh >> (8 * (7 - cnt))) & 0xFFu;
    const uint32_t rem = (uint32_t)zl & 0xFFu;
    zl = (zh << 56) | (zl >> 8);
    zh = (zh >> 8) ^ tb.rem[rem];
    zh ^= ht[b][0];
    zl ^= ht[b][1];
  }
  xh = zh; xl = zl;
}
NFDP_HD void ghash_block(const EspTables& tb, const uint64_t (*ht)[2], uint64_t& xh, uint64_t& xl, const uint32_t be[4]) {
  xh ^= ((uint64_t)be[0] << 32) | be[1];
  xl ^= ((uint64_t)be[2] << 32) | be[3];
  ghash_mul(tb, ht, xh, xl);
}

NFDP_HD uint32_t ld32(const uint8_t* p) { return *reinterpret_cast<const uint32_t*>(p); }   // 4-B aligned
NFDP_HD void st32(uint8_t* p, uint32_t v) { *reinterpret_cast<uint32_t*>(p) = v; }
NFDP_HD uint32_t be16r(const uint8_t* p) { return ((uint32_t)p[0] << 8) | p[1]; }
NFDP_HD uint32_t ipv4_csum20(const uint8_t* h) {   // checksum over a 20-B header with its csum field zero
  uint32_t c = 0;
  for (int o = 0; o < 20; o += 2) c += (o == 10) ? 0u : be16r(h + o);
  c = (c & 0xFFFFu) + (c >> 16);
  c = (c & 0xFFFFu) + (c >> 16);
  return ~c & 0xFFFFu;
}

// GCM keystream / auth over `nw` words of payload: dst[j] = src_word(j) ^ ks, GHASH over the
// ciphertext words.  `src_word(j)` yields payload dword j (LE, memory order); `enc` picks which
// side is the ciphertext.  Returns the tag (4 BE words) in tag[].
template <class SrcWord>
NFDP_HD void gcm_run(const EspTables& tb, const EspSa& sa, uint32_t iv_hi, uint32_t iv_lo, uint32_t seq,
                     uint32_t nw, bool enc, SrcWord src_word, uint8_t* dst, uint32_t tag[4]) {
  const uint32_t salt = bswap32_(sa.salt);
  uint32_t ctr[4] = {salt, iv_hi, iv_lo, 1u}, ek0[4];
  aes_block(tb, sa.rk, sa.nr, ctr, ek0);
  uint64_t xh = 0, xl = 0;
  const uint32_t aad[4] = {sa.spi, seq, 0u, 0u};
  ghash_block(tb, sa.htab, xh, xl, aad);
  // 64-B groups (4 blocks): a lane's payload is read and written a whole cache line at a time,
  // so the line is not evicted between its blocks while 64 lanes stream 64 different packets
  for (uint32_t base = 0; base < nw; base += 16u) {
    uint32_t w[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) w[q] = (base + q < nw) ? src_word(base + q) : 0u;
#pragma unroll
    for (int blk = 0; blk < 4; ++blk) {
      const uint32_t j0 = base + 4u * blk;
      if (j0 >= nw) break;
      ctr[3] = 2u + j0 / 4u;
      uint32_t ks[4];
      aes_block(tb, sa.rk, sa.nr, ctr, ks);
      uint32_t cbe[4] = {0u, 0u, 0u, 0u};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (j0 + q >= nw) break;
        const uint32_t in = w[4 * blk + q];
        const uint32_t out = in ^ bswap32_(ks[q]);
        w[4 * blk + q] = out;
        cbe[q] = bswap32_(enc ? out : in);
      }
      ghash_block(tb, sa.htab, xh, xl, cbe);
    }
#pragma unroll
    for (int q = 0; q < 16; ++q)
      if (base + q < nw) st32(dst + 4 * (base + q), w[q]);
  }
  const uint32_t lens[4] = {0u, 64u, 0u, nw * 32u};   // len(AAD) = 64 bits || len(C) in bits
  ghash_block(tb, sa.htab, xh, xl, lens);
  tag[0] = (uint32_t)(xh >> 32) ^ ek0[0]; tag[1] = (uint32_t)xh ^ ek0[1];
  tag[2] = (uint32_t)(xl >> 32) ^ ek0[2]; tag[3] = (uint32_t)xl ^ ek0[3];
}

NFDP_HD int spd_lookup(const SpdEntry* spd, uint32_t mask, uint32_t dst, uint32_t proto, uint32_t& sa) {
  if (!spd) return kSpdEmpty;
  const uint32_t h = spd_hash(dst, proto);
  for (uint32_t q = 0; q < 8; ++q) {
    const SpdEntry& e = spd[(h + q) & mask];
    if (e.action == kSpdEmpty) return kSpdEmpty;
    if (e.dst_ip == dst && e.proto == proto) { sa = e.sa; return e.action; }
  }
  return kSpdEmpty;
}
NFDP_HD int rxsa_lookup(const RxSaEntry* t, uint32_t mask, uint32_t src, uint32_t dst, uint32_t spi) {
  if (!t) return -1;
  const uint32_t h = rxsa_hash(src, dst, spi);
  for (uint32_t q = 0; q < 8; ++q) {
    const RxSaEntry& e = t[(h + q) & mask];
    if (!e.valid) return -1;
    if (e.src_ip == src && e.dst_ip == dst && e.spi == spi) return e.sa;
  }
  return -1;
}

struct EspBatch {
  const uint8_t* in; uint32_t in_stride; const uint32_t* in_len;
  uint8_t* out; uint32_t out_stride; uint32_t* out_len; uint32_t* status;
  const EspSa* sa; uint32_t n_sa;
  const SpdEntry* spd; uint32_t spd_mask;     // outbound
  const RxSaEntry* rxsa; uint32_t rxsa_mask;  // inbound
  const uint32_t* seq;                        // outbound: sequence number per packet (per-SA counters, host)
  uint32_t* out_sa; uint32_t* out_seq;        // inbound: SA and sequence number (replay window, host)
  uint32_t n;
};

// Outbound: SPD (dst, proto) -> ESP tunnel / transport encapsulation of frame i.
NFDP_HD void esp_encrypt_one(const EspTables& tb, const EspBatch& a, uint32_t i) {
  const uint8_t* f = a.in + (size_t)i * a.in_stride + kClearOff;
  const uint32_t L = a.in_len[i];
  a.out_len[i] = 0;
  if (L + kClearOff + 4u > a.in_stride) { a.status[i] = kEspDrop; return; }   // staging contract broken
  if (L < 34u || be16r(f + 12) != 0x0800u || (f[14] >> 4) != 4u) {
    a.status[i] = kEspBypass;   // not IPv4: not subject to the IPv4 SPD
    return;
  }
  uint32_t s = 0;
  const int act = spd_lookup(a.spd, a.spd_mask, ld32(f + 30), f[23], s);   // dst at slot + 32
  if (act == kSpdDrop) { a.status[i] = kEspDrop; return; }
  if (act != kSpdProtect || s >= a.n_sa || a.sa[s].nr == 0) { a.status[i] = kEspBypass; return; }
  const EspSa& sa = a.sa[s];
  const bool tun = sa.mode == kEspTunnel;
  if (!tun && (f[14] & 0xFu) != 5u) { a.status[i] = kEspDrop; return; }   // transport: no IP options
  const uint32_t poff = tun ? 14u : 34u;       // payload offset in the frame (slot + 16 / + 36)
  const uint32_t plen = L - poff;
  const uint32_t pad = (4u - ((plen + 2u) & 3u)) & 3u;
  const uint32_t ptlen = plen + pad + 2u;
  const uint32_t olen = kEspHdrBytes + ptlen + kEspIcv;
  if (olen + kEspOff > a.out_stride) { a.status[i] = kEspDrop; return; }
  const uint32_t nxt = tun ? 4u : f[23];
  const uint32_t seq = a.seq[i];
  // Sequence number 0 is never sent (RFC 4303 3.3.3: the first packet is 1, the counter never
  // cycles).  The host hands out 0 when an SA's 32-bit space is exhausted or the host SPD does
  // not protect the packet: dropping here is what keeps the GCM nonce (0^32 || seq) unique.
  if (seq == 0u) { a.status[i] = kEspDrop; return; }
  uint8_t* slot = a.out + (size_t)i * a.out_stride;
  // header: 52 bytes from slot + 12 (2 bytes before the frame are zero), 13 aligned dwords
  uint8_t h[52];
  for (int k = 0; k < 52; ++k) h[k] = 0;
  uint8_t* e = h + 2;
  if (tun) {
    for (int k = 0; k < 4; ++k) { e[k] = (sa.dmac_lo >> (8 * k)) & 0xFF; e[6 + k] = (sa.smac_lo >> (8 * k)) & 0xFF; }
    e[4] = sa.dmac_hi & 0xFF; e[5] = sa.dmac_hi >> 8; e[10] = sa.smac_hi & 0xFF; e[11] = sa.smac_hi >> 8;
    e[12] = 0x08; e[13] = 0x00;
    e[14] = 0x45; e[15] = 0; e[18] = (seq >> 8) & 0xFF; e[19] = seq & 0xFF; e[20] = 0x40; e[21] = 0;
    e[22] = 64; e[23] = 50;
    for (int k = 0; k < 4; ++k) { e[26 + k] = (sa.src_ip >> (8 * k)) & 0xFF; e[30 + k] = (sa.dst_ip >> (8 * k)) & 0xFF; }
  } else {
    for (int k = 0; k < 34; ++k) e[k] = f[k];
    e[23] = 50;
  }
  e[16] = ((olen - 14u) >> 8) & 0xFF; e[17] = (olen - 14u) & 0xFF;
  e[24] = 0; e[25] = 0;
  const uint32_t c = ipv4_csum20(e + 14);
  e[24] = (c >> 8) & 0xFF; e[25] = c & 0xFF;
  for (int k = 0; k < 4; ++k) { e[34 + k] = (sa.spi >> (24 - 8 * k)) & 0xFF; e[38 + k] = (seq >> (24 - 8 * k)) & 0xFF; }
  for (int k = 0; k < 4; ++k) e[46 + k] = (seq >> (24 - 8 * k)) & 0xFF;   // IV = 0^32 || seq
  for (int k = 0; k < 13; ++k)
    st32(slot + 12 + 4 * k, (uint32_t)h[4 * k] | ((uint32_t)h[4 * k + 1] << 8) | ((uint32_t)h[4 * k + 2] << 16) |
                               ((uint32_t)h[4 * k + 3] << 24));
  const uint8_t* p = f + poff;   // 4-B aligned
  auto word = [&](uint32_t j) -> uint32_t {
    uint32_t w = (4 * j < plen) ? ld32(p + 4 * j) : 0u;
    if (4 * j + 4 > plen) {
      for (uint32_t q = 0; q < 4; ++q) {
        const uint32_t k = 4 * j + q;
        if (k < plen) continue;
        const uint32_t v = k < plen + pad ? (k - plen + 1u) : (k == plen + pad ? pad : nxt);
        w = (w & ~(0xFFu << (8 * q))) | (v << (8 * q));
      }
    }
    return w;
  };
  uint32_t tag[4];
  gcm_run(tb, sa, 0u, seq, seq, ptlen / 4u, true, word, slot + 64, tag);
  for (int q = 0; q < 4; ++q) st32(slot + 64 + ptlen + 4 * q, bswap32_(tag[q]));
  a.out_len[i] = olen;
  a.status[i] = kEspDone;
}

// Inbound: (src, dst, SPI) -> SA, authenticate + decrypt, strip the outer header (tunnel) or the
// ESP header / trailer (transport).  The decrypted frame sits at out slot + kClearOff.
NFDP_HD void esp_decrypt_one(const EspTables& tb, const EspBatch& a, uint32_t i) {
  const uint8_t* slot_in = a.in + (size_t)i * a.in_stride;
  const uint8_t* f = slot_in + kEspOff;
  const uint32_t L = a.in_len[i];
  a.out_len[i] = 0;
  a.out_sa[i] = 0xFFFFFFFFu;
  a.out_seq[i] = 0;
  if (L < (uint32_t)(kEspHdrBytes + kEspIcv + 4) || L + kEspOff > a.in_stride || be16r(f + 12) != 0x0800u ||
      f[14] != 0x45u || f[23] != 50u) {
    a.status[i] = kEspDrop;
    return;
  }
  const uint32_t src = ld32(slot_in + 40), dst = ld32(slot_in + 44);
  const uint32_t spi = bswap32_(ld32(slot_in + 48)), seq = bswap32_(ld32(slot_in + 52));
  const int s = rxsa_lookup(a.rxsa, a.rxsa_mask, src, dst, spi);
  if (s < 0 || (uint32_t)s >= a.n_sa || a.sa[s].nr == 0) { a.status[i] = kEspNoSa; return; }
  const EspSa& sa = a.sa[s];
  const uint32_t ctlen = L - kEspHdrBytes - kEspIcv;
  if (ctlen & 3u) { a.status[i] = kEspDrop; return; }
  const bool tun = sa.mode == kEspTunnel;
  uint8_t* slot = a.out + (size_t)i * a.out_stride;
  const uint32_t poff = tun ? 14u : 34u;
  if (kClearOff + poff + ctlen > a.out_stride) { a.status[i] = kEspDrop; return; }
  const uint32_t iv_hi = bswap32_(ld32(slot_in + 56)), iv_lo = bswap32_(ld32(slot_in + 60));
  const uint8_t* c = slot_in + 64;
  uint32_t last = 0;
  auto word = [&](uint32_t j) -> uint32_t { return ld32(c + 4 * j); };
  uint32_t tag[4];
  gcm_run(tb, sa, iv_hi, iv_lo, seq, ctlen / 4u, false, word, slot + kClearOff + poff, tag);
  bool ok = true;
  for (int q = 0; q < 4; ++q) ok = ok && bswap32_(ld32(c + ctlen + 4 * q)) == tag[q];
  last = ld32(slot + kClearOff + poff + ctlen - 4);
  const uint32_t padl = (last >> 16) & 0xFFu, nxt = last >> 24;
  if (!ok || padl + 2u > ctlen || (tun && nxt != 4u)) { a.status[i] = kEspAuthFail; return; }
  const uint32_t ilen = ctlen - 2u - padl;   // inner IP packet (tunnel) / L4 payload (transport)
  // header dwords before the payload: slot + 0 .. slot + kClearOff + poff
  uint8_t h[36];
  for (int k = 0; k < 36; ++k) h[k] = 0;
  uint8_t* e = h + kClearOff;
  for (int k = 0; k < 12; ++k) e[k] = f[k];
  e[12] = 0x08; e[13] = 0x00;
  if (!tun) {
    for (int k = 14; k < 34; ++k) e[k] = f[k];
    e[23] = (uint8_t)nxt;
    e[16] = ((20u + ilen) >> 8) & 0xFF; e[17] = (20u + ilen) & 0xFF;
    e[24] = 0; e[25] = 0;
    const uint32_t cs = ipv4_csum20(e + 14);
    e[24] = (cs >> 8) & 0xFF; e[25] = cs & 0xFF;
  }
  const uint32_t hw = (kClearOff + poff) / 4u;   // 4 (tunnel) or 9 (transport) dwords
  for (uint32_t k = 0; k < hw; ++k)
    st32(slot + 4 * k, (uint32_t)h[4 * k] | ((uint32_t)h[4 * k + 1] << 8) | ((uint32_t)h[4 * k + 2] << 16) |
                          ((uint32_t)h[4 * k + 3] << 24));
  a.out_len[i] = poff + ilen;
  a.out_sa[i] = (uint32_t)s;
  a.out_seq[i] = seq;
  a.status[i] = kEspDone;
}

}  // namespace nfdp
