// shard_cpu.cpp — scalar CPU twins of the sharded stage kernels (gloo multi-process tests and
// the bit-exact oracle for the multi-GPU path).  Slot positions are assigned in packet order;
// the GPU assigns them with wave-aggregated atomics, so tests compare per-packet outcomes, not
// segment layouts.
#include <cstring>

#include "shard.h"

namespace nfdp {

void ingress_cpu(const IngressArgs& a) {
  const size_t seg = desc_seg_bytes(a.g.cap_desc);
  for (uint32_t i = 0; i < a.n; ++i) {
    uint32_t d[kSlotDwords];
    std::memcpy(d, reinterpret_cast<const uint8_t*>(a.pkts) + (size_t)i * kSlotBytes, kSlotBytes);
    Parsed p;
    IngressState st;
    ingress_stage(a.t, d, a.inmeta[i], p, st);
    const uint32_t h = toeplitz_scalar(st.key, a.t.rss_key);
    const int acl = acl_rule_scalar(a.t, p, st);
    uint32_t ref = kRefNone;
    if (!st.reason && p.ipv4) {
      const uint32_t owner = owner_of(h, a.g.nranks);
      const uint32_t pos = a.cnt[owner]++;
      if (pos < a.g.cap_desc) {
        const uint32_t dsc[8] = {st.key.src_ip, st.key.dst_ip, st.key.ports, st.key.meta, st.wire_len, 0, 0, 0};
        std::memcpy(a.send_desc + owner * seg + 32 * (1 + (size_t)pos), dsc, 32);
        ref = (owner << 24) | pos;
      } else {
        ref = kRefOverflow;
      }
    }
    a.ref[i] = ref;
    a.aux[i] = (uint32_t)(acl + 1) | ((h & 7u) << 16);
  }
  for (uint32_t o = 0; o < a.g.nranks; ++o) {
    const uint32_t hdr[4] = {a.cnt[o] < a.g.cap_desc ? a.cnt[o] : a.g.cap_desc, a.g.cap_desc, 0, 0};
    std::memcpy(a.send_desc + o * seg, hdr, 16);
  }
}

void owner_cpu(const OwnerArgs& a) {
  const size_t seg = desc_seg_bytes(a.g.cap_desc), vseg = verdict_seg_bytes(a.g.cap_desc);
  for (uint32_t s = 0; s < a.g.nranks; ++s) {
    uint32_t hdr[4];
    std::memcpy(hdr, a.recv_desc + s * seg, 16);
    std::memcpy(a.send_verdict + s * vseg, hdr, 16);
    for (uint32_t j = 0; j < hdr[0] && j < a.g.cap_desc; ++j) {
      uint32_t dsc[8];
      std::memcpy(dsc, a.recv_desc + s * seg + 32 * (1 + (size_t)j), 32);
      const FlowKey k{dsc[0], dsc[1], dsc[2], dsc[3]};
      const uint32_t wlen = dsc[4];
      const uint32_t h = toeplitz_scalar(k, a.t.rss_key);
      const int64_t slot = flow_lookup(a.t, k, h);
      uint32_t out[4] = {0, 0, 0, 0};
      if (slot >= 0) {
        std::memcpy(out, &a.t.flows[slot].act, 12);
        out[3] = 1;
        if (a.flow_ctr) a.flow_ctr[slot] += ctr_inc(wlen);
      }
      std::memcpy(a.send_verdict + s * vseg + 16 * (1 + (size_t)j), out, 16);
    }
  }
}

void apply_cpu(const ApplyArgs& a) {
  const size_t dseg = verdict_seg_bytes(a.g.cap_desc);
  const size_t pseg = pkt_seg_bytes(a.g.cap_pkt);
  for (uint32_t i = 0; i < a.n; ++i) {
    uint32_t d[kSlotDwords];
    std::memcpy(d, reinterpret_cast<const uint8_t*>(a.pkts) + (size_t)i * kSlotBytes, kSlotBytes);
    Parsed p;
    IngressState st;
    ingress_stage(a.t, d, a.inmeta[i], p, st);
    bool hit = false;
    FlowAction act = {};
    const uint32_t ref = a.ref[i];
    if (ref == kRefOverflow) {
      st.reason = st.reason ? st.reason : kOverflow;
    } else if (ref != kRefNone) {
      uint32_t v[4];
      std::memcpy(v, a.recv_verdict + (ref >> 24) * dseg + 16 * (1 + (size_t)(ref & 0xFFFFFFu)), 16);
      hit = v[3] == 1u;
      act.chain_id = v[0] & 0xFFFFu; act.out_port = v[0] >> 16; act.nat_ip = v[1];
      act.nat_port = v[2] & 0xFFFFu; act.vlan = v[2] >> 16;
    }
    const EgressDecision e = chain_stage(a.t, p, st, hit, act, (int)(a.aux[i] & 0xFFFFu) - 1, a.aux[i] >> 16);
    uint32_t eg = a.g.rank;
    if (!e.reason) eg = a.t.ports[e.out_port].gpu;
    const bool remote = !e.reason && eg != a.g.rank && eg < a.g.nranks;
    uint32_t o[kSlotDwords];
    emit(p, e.tci, e.push != 0, o);
    const uint32_t olen = egress_len(p, e);
    uint32_t reason = e.reason;
    uint32_t pos = 0;
    if (remote) {
      pos = a.pcnt[eg]++;
      if (pos >= a.g.cap_pkt) reason = kOverflow;
    }
    if (remote && reason == kOk) {
      uint8_t* segp = a.send_pkt + eg * pseg;
      std::memcpy(segp + 64 + (size_t)pos * 64, o, 64);
      const uint32_t m = make_meta(e.out_port, olen, kOk, e.xhdr != 0);
      std::memcpy(segp + pkt_meta_off(a.g.cap_pkt) + 4 * (size_t)pos, &m, 4);
      a.out_meta[i] = make_meta(e.out_port, olen, kRemote);
    } else {
      std::memcpy(reinterpret_cast<uint8_t*>(a.out) + (size_t)i * 64, o, 64);
      a.out_meta[i] = make_meta(reason == kOverflow ? kPortNone : e.out_port, reason == e.reason ? olen : 0u, reason, !reason && e.xhdr, !reason && e.flood);
    }
    if (st.in_port < (uint32_t)kMaxPorts) a.port_ctr[2 * st.in_port] += ctr_inc(st.wire_len);
    if (reason) a.drop_ctr[reason & (kNumReasons - 1)] += 1;
    else if (!remote) a.port_ctr[2 * e.out_port + 1] += ctr_inc(olen);
  }
  for (uint32_t e = 0; e < a.g.nranks; ++e) {
    const uint32_t c = a.pcnt[e] < a.g.cap_pkt ? a.pcnt[e] : a.g.cap_pkt;
    const uint32_t hdr[4] = {c, a.g.cap_pkt, 0, 0};
    std::memcpy(a.send_pkt + e * pseg, hdr, 16);
  }
}

void egress_cpu(const EgressArgs& a) {
  const size_t pseg = pkt_seg_bytes(a.g.cap_pkt);
  for (uint32_t s = 0; s < a.g.nranks; ++s) {
    if (s == a.g.rank) continue;
    const uint8_t* segp = a.recv_pkt + s * pseg;
    uint32_t count;
    std::memcpy(&count, segp, 4);
    for (uint32_t j = 0; j < count && j < a.g.cap_pkt; ++j) {
      uint32_t m;
      std::memcpy(&m, segp + pkt_meta_off(a.g.cap_pkt) + 4 * (size_t)j, 4);
      const uint32_t port = meta_port(m), len = meta_len(m);
      if (port < (uint32_t)kMaxPorts) a.port_ctr[2 * port + 1] += ctr_inc(len);
    }
  }
}

}  // namespace nfdp
