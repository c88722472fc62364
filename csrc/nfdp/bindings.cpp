// bindings.cpp — pybind11 module `_nfdp`: the Python control plane's handle on the native data
// plane.  Buffers cross the boundary as raw addresses (torch HBM tensors or numpy host arrays),
// so no copies and no torch headers are involved; the HIP stream is passed as an integer
// (torch.cuda.current_stream().cuda_stream).
#include <algorithm>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "host.h"
#include "iox.h"
#include "ipsec.h"
#include "pktio.h"
#include "ring.h"
#include "shard.h"
#include "trafgen.h"
#include "trafgen_pkt.h"

namespace py = pybind11;
using namespace nfdp;

namespace {

template <typename T>
T* ptr(const py::dict& d, const char* k) {
  if (!d.contains(k)) return nullptr;
  py::object o = d[k];
  if (o.is_none()) return nullptr;
  return reinterpret_cast<T*>(o.cast<uintptr_t>());
}
template <typename T>
T val(const py::dict& d, const char* k, T def) {
  if (!d.contains(k)) return def;
  return d[k].cast<T>();
}

TablesView tables_from(const py::dict& d);
// IPv6 ACL tiles of a fused launch (tables dict: acl6_wfrag / acl6_cinit / acl6_tiles)
void acl6_from(FusedLaunch& f, const py::dict& d) {
  f.acl6_wfrag = ptr<const void>(d, "acl6_wfrag");
  f.acl6_cinit = ptr<const void>(d, "acl6_cinit");
  f.acl6_tiles = val<uint32_t>(d, "acl6_tiles", 0);
}

TablesView tables_from(const py::dict& d) {
  TablesView t{};
  t.ports = ptr<const PortEntry>(d, "ports");
  t.chains = ptr<const ChainEntry>(d, "chains");
  t.n_chains = val<uint32_t>(d, "n_chains", 0);
  t.flows = ptr<const FlowSlot>(d, "flows");
  t.bucket_mask = val<uint32_t>(d, "bucket_mask", 0);
  t.macs = ptr<const MacEntry>(d, "macs");
  t.mac_mask = val<uint32_t>(d, "mac_mask", 0);
  t.rss_key = ptr<const uint8_t>(d, "rss_key");
  t.acl_value = ptr<const uint32_t>(d, "acl_value");
  t.acl_mask = ptr<const uint32_t>(d, "acl_mask");
  t.acl_permit = ptr<const uint8_t>(d, "acl_permit");
  t.n_acl = val<uint32_t>(d, "n_acl", 0);
  t.acl_default_permit = val<uint32_t>(d, "acl_default_permit", 1);
  t.lag_members = d.contains("lag_members") ? ptr<const uint16_t>(d, "lag_members") : nullptr;
  t.n_lag_groups = val<uint32_t>(d, "n_lag_groups", 0);
  t.flood = ptr<const uint16_t>(d, "flood");
  t.n_flood = t.flood ? val<uint32_t>(d, "n_flood", 0) : 0u;
  t.lpm6 = ptr<const Lpm6Entry>(d, "lpm6");
  t.lpm6_mask = t.lpm6 ? val<uint32_t>(d, "lpm6_mask", 0) : 0u;
  t.lpm6_lens = ptr<const uint8_t>(d, "lpm6_lens");
  t.n_lpm6_lens = t.lpm6_lens ? val<uint32_t>(d, "n_lpm6_lens", 0) : 0u;
  t.flow6_on = val<uint32_t>(d, "flow6_on", 0);
  t.acl6_value = ptr<const uint32_t>(d, "acl6_value");
  t.acl6_mask = ptr<const uint32_t>(d, "acl6_mask");
  t.n_acl6 = (t.acl6_value && t.acl6_mask) ? val<uint32_t>(d, "n_acl6", 0) : 0u;
  if (t.n_acl6 > 4096) throw std::invalid_argument("at most 4096 IPv6 ACL rules");
  if (t.n_acl6 && !t.acl_permit) throw std::invalid_argument("n_acl6 > 0 but acl_permit missing");
  if (t.lpm6 && ((t.lpm6_mask + 1) & t.lpm6_mask)) throw std::invalid_argument("lpm6 table size must be a power of two");
  if (t.n_lpm6_lens > 129) throw std::invalid_argument("at most 129 IPv6 prefix lengths");
  t.lpm24 = ptr<const uint32_t>(d, "lpm24");
  t.lpm8 = ptr<const uint32_t>(d, "lpm8");
  t.n_lpm8 = t.lpm8 ? val<uint32_t>(d, "n_lpm8", 0) : 0u;
  t.nexthops = ptr<const NextHop>(d, "nexthops");
  t.n_nexthops = t.nexthops ? val<uint32_t>(d, "n_nexthops", 0) : 0u;
  t.ecmp = ptr<const uint16_t>(d, "ecmp");
  t.n_ecmp = t.ecmp ? val<uint32_t>(d, "n_ecmp", 0) : 0u;
  t.tunnels = ptr<const TunnelEntry>(d, "tunnels");
  t.n_tunnels = t.tunnels ? val<uint32_t>(d, "n_tunnels", 0) : 0u;
  t.tunnels6 = ptr<const Tunnel6Entry>(d, "tunnels6");
  t.n_tunnels6 = t.tunnels6 ? val<uint32_t>(d, "n_tunnels6", 0) : 0u;
  t.vtep6_fold = val<uint32_t>(d, "vtep6_fold", 0);
  t.terms = ptr<const TermEntry>(d, "terms");
  t.term_mask = t.terms ? val<uint32_t>(d, "term_mask", 0) : 0u;
  if (t.terms && ((t.term_mask + 1) & t.term_mask)) throw std::invalid_argument("term table size must be a power of two");
  t.terms6 = ptr<const Term6Entry>(d, "terms6");
  t.term6_mask = t.terms6 ? val<uint32_t>(d, "term6_mask", 0) : 0u;
  if (t.terms6 && ((t.term6_mask + 1) & t.term6_mask)) throw std::invalid_argument("term6 table size must be a power of two");
  if (d.contains("vtep6")) {
    const auto v = d["vtep6"].cast<std::vector<uint32_t>>();
    if (v.size() != 4) throw std::invalid_argument("vtep6: 4 raw words");
    for (int k = 0; k < 4; ++k) t.vtep6[k] = v[k];
  }
  t.vmmac = ptr<const VmMacEntry>(d, "vmmac");
  t.vmmac_mask = t.vmmac ? val<uint32_t>(d, "vmmac_mask", 0) : 0u;
  if (t.vmmac && ((t.vmmac_mask + 1) & t.vmmac_mask)) throw std::invalid_argument("vmmac table size must be a power of two");
  if (t.n_lag_groups && !t.lag_members) throw std::invalid_argument("n_lag_groups > 0 but lag_members missing");
  if (!t.ports || !t.chains || !t.flows || !t.rss_key)
    throw std::invalid_argument("tables dict is missing a required buffer");
  if (t.n_acl && (!t.acl_value || !t.acl_mask || !t.acl_permit))
    throw std::invalid_argument("n_acl > 0 but ACL buffers missing");
  return t;
}

// Side outputs (replicas + learn events): a dict of buffer addresses and capacities, or None.
SideOut side_from(const py::object& o) {
  SideOut so{};
  if (o.is_none()) return so;
  const py::dict d = o.cast<py::dict>();
  so.rep_hdr = ptr<uint32_t>(d, "rep_hdr"); so.rep_meta = ptr<uint32_t>(d, "rep_meta");
  so.rep_src = ptr<uint32_t>(d, "rep_src"); so.cap_rep = val<uint32_t>(d, "cap_rep", 0);
  so.learn = ptr<uint32_t>(d, "learn"); so.cap_learn = val<uint32_t>(d, "cap_learn", 0);
  so.cnt = ptr<uint32_t>(d, "cnt");
  so.list = ptr<uint32_t>(d, "list"); so.cap_list = val<uint32_t>(d, "cap_list", 0);
  so.xhdr = ptr<uint32_t>(d, "xhdr");
  so.blk_cnt = ptr<uint32_t>(d, "blk_cnt");              // per-workgroup regions (fused kernel)
  so.nblk = so.blk_cnt ? val<uint32_t>(d, "blk_max", 0) : 0u;   // blk_cnt entries (the launcher's grid cap)
  if (!so.cnt) throw std::invalid_argument("side outputs need a 'cnt' buffer (4 x u32)");
  if (so.cap_rep && (!so.rep_hdr || !so.rep_meta || !so.rep_src)) throw std::invalid_argument("side: replica buffers missing");
  if (so.cap_learn && !so.learn) throw std::invalid_argument("side: learn buffer missing");
  return so;
}

// ESP batch (ipsec.h EspBatch) from a dict of buffer addresses and sizes.
EspBatch esp_from(const py::dict& d) {
  EspBatch a{};
  a.in = ptr<const uint8_t>(d, "in"); a.in_stride = val<uint32_t>(d, "in_stride", 0);
  a.in_len = ptr<const uint32_t>(d, "in_len");
  a.out = ptr<uint8_t>(d, "out"); a.out_stride = val<uint32_t>(d, "out_stride", 0);
  a.out_len = ptr<uint32_t>(d, "out_len"); a.status = ptr<uint32_t>(d, "status");
  a.sa = ptr<const EspSa>(d, "sa"); a.n_sa = val<uint32_t>(d, "n_sa", 0);
  a.spd = ptr<const SpdEntry>(d, "spd"); a.spd_mask = val<uint32_t>(d, "spd_mask", 0);
  a.rxsa = ptr<const RxSaEntry>(d, "rxsa"); a.rxsa_mask = val<uint32_t>(d, "rxsa_mask", 0);
  a.seq = ptr<const uint32_t>(d, "seq");
  a.out_sa = ptr<uint32_t>(d, "out_sa"); a.out_seq = ptr<uint32_t>(d, "out_seq");
  a.n = val<uint32_t>(d, "n", 0);
  if (a.n && (!a.in || !a.out || !a.in_len || !a.out_len || !a.status || !a.sa))
    throw std::invalid_argument("esp batch: missing buffer");
  if ((a.in_stride & 15u) || (a.out_stride & 15u) || a.in_stride < 64u || a.out_stride < 128u)
    throw std::invalid_argument("esp batch: strides must be multiples of 16 (>= 64 in, >= 128 out)");
  if (a.spd && ((a.spd_mask + 1) & a.spd_mask)) throw std::invalid_argument("esp: SPD size must be a power of two");
  if (a.rxsa && ((a.rxsa_mask + 1) & a.rxsa_mask)) throw std::invalid_argument("esp: RX SA size must be a power of two");
  if (a.n_sa > (uint32_t)kEspMaxSa) throw std::invalid_argument("esp: too many SAs");
  return a;
}

void check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

using U32Arr = py::array_t<uint32_t, py::array::c_style | py::array::forcecast>;

}  // namespace

PYBIND11_MODULE(_nfdp, m) {
  m.doc() = "MI355X network-function data plane (HIP/CDNA4 kernels + host control structures)";
  m.attr("SLOT_BYTES") = kSlotBytes;
  m.attr("MAX_PORTS") = kMaxPorts;
  m.attr("BUCKET_SLOTS") = kBucketSlots;
  m.attr("PORT_NONE") = kPortNone;
  m.attr("PORT_PUNT") = kPortPunt;
  m.attr("NUM_REASONS") = (int)kNumReasons;
  m.attr("MAX_FRAME") = kMaxFrame;
  m.attr("FLOOD_WAYS") = kFloodWays;
  m.attr("ENCAP_BYTES") = kEncapBytes;
  m.attr("ENCAP6_BYTES") = kEncap6Bytes;
  m.attr("XHDR_BYTES") = kXhdrBytes;
  m.attr("PORT_TUNNEL6") = (uint32_t)kPortTunnel6;
  m.def("vtep6_fold", [](uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3) { return vtep6_fold(a0, a1, a2, a3); });
  // outer headers of a tunnel entry (32-B IPv4-underlay or 64-B IPv6-underlay entry bytes)
  m.def("make_outer", [](py::bytes te_raw, uint32_t inner_len, uint32_t hash) {
    std::string s = te_raw;
    uint32_t x[kXhdrBytes / 4] = {};
    if (s.size() == sizeof(TunnelEntry)) {
      TunnelEntry te;
      std::memcpy(&te, s.data(), sizeof(te));
      make_outer(te, inner_len, hash, x);
      return py::bytes(reinterpret_cast<const char*>(x), kEncapBytes);
    }
    if (s.size() != sizeof(Tunnel6Entry)) throw std::invalid_argument("tunnel entry must be 32 (IPv4) or 64 (IPv6) bytes");
    Tunnel6Entry te;
    std::memcpy(&te, s.data(), sizeof(te));
    make_outer6(te, inner_len, hash, x);
    return py::bytes(reinterpret_cast<const char*>(x), kEncap6Bytes);
  });

  py::class_<FlowTableHost>(m, "FlowTable")
      .def(py::init([](uint32_t nb, py::bytes rss) {
             std::string s = rss;
             return new FlowTableHost(nb, std::vector<uint8_t>(s.begin(), s.end()));
           }),
           py::arg("nbuckets"), py::arg("rss_key"))
      .def_property_readonly("nbuckets", &FlowTableHost::nbuckets)
      .def_property_readonly("mask", &FlowTableHost::mask)
      .def("__len__", &FlowTableHost::size)
      .def("hash", [](const FlowTableHost& t, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
        return t.hash(FlowKey{a, b, c, d});
      })
      .def("insert", [](FlowTableHost& t, py::tuple k, py::tuple v) {
        FlowKey key{k[0].cast<uint32_t>(), k[1].cast<uint32_t>(), k[2].cast<uint32_t>(), k[3].cast<uint32_t>()};
        const uint32_t w0 = v[0].cast<uint32_t>(), w1 = v[1].cast<uint32_t>(), w2 = v[2].cast<uint32_t>(), w3 = v[3].cast<uint32_t>();
        FlowAction a;
        a.chain_id = w0 & 0xFFFF; a.out_port = w0 >> 16; a.nat_ip = w1;
        a.nat_port = w2 & 0xFFFF; a.vlan = w2 >> 16; a.flow_id = w3;
        return t.insert(key, a);
      })
      .def("insert_many", [](FlowTableHost& t, U32Arr keys, U32Arr vals) {
        if (keys.ndim() != 2 || keys.shape(1) != 4 || vals.ndim() != 2 || vals.shape(1) != 4 ||
            keys.shape(0) != vals.shape(0))
          throw std::invalid_argument("insert_many expects [n,4] uint32 keys and values");
        const size_t n = keys.shape(0);
        py::array_t<int64_t> slots(n);
        auto k = keys.unchecked<2>();
        auto v = vals.unchecked<2>();
        auto o = slots.mutable_unchecked<1>();
        for (size_t i = 0; i < n; ++i) {
          FlowKey key{k(i, 0), k(i, 1), k(i, 2), k(i, 3)};
          FlowAction a;
          a.chain_id = v(i, 0) & 0xFFFF; a.out_port = v(i, 0) >> 16; a.nat_ip = v(i, 1);
          a.nat_port = v(i, 2) & 0xFFFF; a.vlan = v(i, 2) >> 16; a.flow_id = v(i, 3);
          o(i) = t.insert(key, a);
        }
        return slots;
      })
      .def("erase_many", [](FlowTableHost& t, U32Arr keys) {
        if (keys.ndim() != 2 || keys.shape(1) != 4) throw std::invalid_argument("erase_many expects [n,4] uint32 keys");
        auto k = keys.unchecked<2>();
        size_t n = 0;
        for (py::ssize_t i = 0; i < keys.shape(0); ++i) n += t.erase(FlowKey{k(i, 0), k(i, 1), k(i, 2), k(i, 3)}) ? 1 : 0;
        return n;
      })
      .def("erase", [](FlowTableHost& t, py::tuple k) {
        return t.erase(FlowKey{k[0].cast<uint32_t>(), k[1].cast<uint32_t>(), k[2].cast<uint32_t>(), k[3].cast<uint32_t>()});
      })
      .def("find", [](const FlowTableHost& t, py::tuple k) {
        return t.find(FlowKey{k[0].cast<uint32_t>(), k[1].cast<uint32_t>(), k[2].cast<uint32_t>(), k[3].cast<uint32_t>()});
      })
      .def("slots", [](const FlowTableHost& t) {
        // [nbuckets*4, 8] uint32: key (4 words, meta |= 0x100 when used) + action (4 words)
        auto& v = t.slots();
        return py::array_t<uint32_t>({(py::ssize_t)v.size(), (py::ssize_t)8}, reinterpret_cast<const uint32_t*>(v.data()));
      })
      .def("take_dirty", [](FlowTableHost& t) {
        auto v = t.take_dirty();
        return py::array_t<uint32_t>(v.size(), v.data());
      })
      .def("take_moves", &FlowTableHost::take_moves)
      .def("clear_dirty", &FlowTableHost::clear_dirty);

  m.def("deferred_host_unmaps", &deferred_host_unmaps,
        "zero-copy host regions waiting for every ring grid of the process to stop before they unregister");
  m.def("toeplitz", [](U32Arr keys, py::bytes rss) {
    std::string s = rss;
    if (s.size() < 20) throw std::invalid_argument("rss key must be >= 20 bytes");
    if (keys.ndim() != 2 || keys.shape(1) != 4) throw std::invalid_argument("keys must be [n,4]");
    const size_t n = keys.shape(0);
    py::array_t<uint32_t> out(n);
    auto k = keys.unchecked<2>();
    auto o = out.mutable_unchecked<1>();
    for (size_t i = 0; i < n; ++i)
      o(i) = toeplitz_scalar(FlowKey{k(i, 0), k(i, 1), k(i, 2), k(i, 3)}, reinterpret_cast<const uint8_t*>(s.data()));
    return out;
  });
  m.def("table_hash", [](uint32_t h, uint32_t mask) {
    TableHash t = table_hash(h, mask);
    return py::make_tuple(t.b1, t.b2);
  });
  m.def("owner_of", &owner_of);
  // IPv6 FIB (nfdp.h lpm6_lookup): routes [n, 6] = (a0..a3 host-order masked prefix, plen, result)
  // -> open-addressing table [slots, 8] u32 (<= 50 % load, every entry within kLpm6Probe of its
  // home slot) + the distinct lengths, longest first.
  m.def("build_lpm6", [](U32Arr routes) {
    if (routes.ndim() != 2 || routes.shape(1) != 6) throw std::invalid_argument("build_lpm6 expects [n,6] uint32");
    const size_t n = routes.shape(0);
    auto r = routes.unchecked<2>();
    std::vector<uint8_t> lens;
    bool seen[129] = {};
    for (size_t i = 0; i < n; ++i) {
      if (r(i, 4) > 128) throw std::invalid_argument("IPv6 prefix length > 128");
      if (!seen[r(i, 4)]) { seen[r(i, 4)] = true; lens.push_back((uint8_t)r(i, 4)); }
    }
    std::sort(lens.begin(), lens.end(), [](uint8_t x, uint8_t y) { return x > y; });
    size_t slots = 16;
    while (slots < 2 * n) slots <<= 1;
    std::vector<Lpm6Entry> tab;
    for (;;) {
      tab.assign(slots, Lpm6Entry{{0, 0, 0, 0}, kLpm6Empty, 0, {0, 0}});
      bool ok = true;
      for (size_t i = 0; i < n && ok; ++i) {
        const uint32_t a[4] = {r(i, 0), r(i, 1), r(i, 2), r(i, 3)};
        const uint32_t h = lpm6_hash(a[0], a[1], a[2], a[3], r(i, 4)) & (uint32_t)(slots - 1);
        ok = false;
        for (int probe = 0; probe < kLpm6Probe; ++probe) {
          Lpm6Entry& e = tab[(h + probe) & (slots - 1)];
          if (e.plen == kLpm6Empty || (e.plen == r(i, 4) && e.a[0] == a[0] && e.a[1] == a[1] && e.a[2] == a[2] && e.a[3] == a[3])) {
            for (int w = 0; w < 4; ++w) e.a[w] = a[w];
            e.plen = r(i, 4); e.result = r(i, 5);
            ok = true;
            break;
          }
        }
      }
      if (ok) break;
      slots <<= 1;
    }
    py::array_t<uint32_t> t({(py::ssize_t)slots, (py::ssize_t)8});
    std::memcpy(t.mutable_data(), tab.data(), slots * sizeof(Lpm6Entry));
    py::array_t<uint8_t> l((py::ssize_t)std::max<size_t>(lens.size(), 1));
    if (!lens.empty()) std::memcpy(l.mutable_data(), lens.data(), lens.size());
    else l.mutable_data()[0] = 0;
    return py::make_tuple(t, l, (uint32_t)lens.size());
  });
  m.def("build_acl_frags", [](U32Arr value, U32Arr mask) {
    if (value.ndim() != 2 || value.shape(1) != 4 || mask.ndim() != 2 || mask.shape(1) != 4 ||
        value.shape(0) != mask.shape(0))
      throw std::invalid_argument("ACL value/mask must be [n,4] uint32");
    AclFrags f = build_acl_frags(value.data(), mask.data(), (uint32_t)value.shape(0));
    return py::make_tuple(py::array_t<int8_t>(f.wfrag.size(), f.wfrag.data()),
                          py::array_t<int32_t>(f.cinit.size(), f.cinit.data()), f.tiles);
  });
  m.def("build_acl6_frags", [](U32Arr value, U32Arr mask) {
    if (value.ndim() != 2 || value.shape(1) != 12 || mask.ndim() != 2 || mask.shape(1) != 12 ||
        value.shape(0) != mask.shape(0))
      throw std::invalid_argument("IPv6 ACL value/mask must be [n,12] uint32");
    AclFrags f = build_acl6_frags(value.data(), mask.data(), (uint32_t)value.shape(0));
    return py::make_tuple(py::array_t<int8_t>(f.wfrag.size(), f.wfrag.data()),
                          py::array_t<int32_t>(f.cinit.size(), f.cinit.data()), f.tiles);
  });
  m.def("fold6", [](uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3) { return fold6(a0, a1, a2, a3); });
  m.def("build_toeplitz_frags", [](py::bytes rss) {
    std::string s = rss;
    if (s.size() < 20) throw std::invalid_argument("rss key must be >= 20 bytes");
    auto v = build_toeplitz_frags(reinterpret_cast<const uint8_t*>(s.data()));
    return py::array_t<int8_t>(v.size(), v.data());
  });
  m.def("build_toeplitz_table", [](py::bytes rss) {
    std::string s = rss;
    if (s.size() < 20) throw std::invalid_argument("rss key too short");
    auto v = build_toeplitz_table(reinterpret_cast<const uint8_t*>(s.data()));
    return py::array_t<uint32_t>(v.size(), v.data());
  });

  m.def("oracle_run", [](py::dict tables, uintptr_t pkts, uintptr_t inmeta, uint32_t n, uintptr_t out,
                         uintptr_t out_meta, uintptr_t flow_ctr, uintptr_t port_ctr, uintptr_t drop_ctr,
                         uintptr_t hashes, uintptr_t acl, py::object side, uintptr_t hop_state) {
    TablesView t = tables_from(tables);
    SideOut so = side_from(side);
    so.blk_cnt = nullptr;       // standalone side pass / oracle: one flat list
    py::gil_scoped_release nogil;
    oracle_run(t, reinterpret_cast<const uint32_t*>(pkts), reinterpret_cast<const uint32_t*>(inmeta), n,
               reinterpret_cast<uint32_t*>(out), reinterpret_cast<uint32_t*>(out_meta),
               reinterpret_cast<uint64_t*>(flow_ctr), reinterpret_cast<uint64_t*>(port_ctr),
               reinterpret_cast<uint64_t*>(drop_ctr), reinterpret_cast<uint32_t*>(hashes),
               reinterpret_cast<int32_t*>(acl), so.cnt ? &so : nullptr, reinterpret_cast<HopState*>(hop_state));
  }, py::arg("tables"), py::arg("pkts"), py::arg("inmeta"), py::arg("n"), py::arg("out"), py::arg("out_meta"),
     py::arg("flow_ctr"), py::arg("port_ctr"), py::arg("drop_ctr"), py::arg("hashes"), py::arg("acl"),
     py::arg("side") = py::none(), py::arg("hop_state") = 0);
  // SFC hop pipeline across GPUs (split chains): the oracle's resume, the GPU hand-off and resume
  m.def("oracle_resume", [](py::dict tables, uintptr_t hdr, uintptr_t state, uint32_t n, uintptr_t out,
                            uintptr_t out_meta, uintptr_t out_state, uintptr_t port_ctr, uintptr_t drop_ctr) {
    const TablesView t = tables_from(tables);
    py::gil_scoped_release nogil;
    oracle_resume(t, reinterpret_cast<const uint32_t*>(hdr), reinterpret_cast<const HopState*>(state), n,
                  reinterpret_cast<uint32_t*>(out), reinterpret_cast<uint32_t*>(out_meta),
                  reinterpret_cast<HopState*>(out_state), reinterpret_cast<uint64_t*>(port_ctr),
                  reinterpret_cast<uint64_t*>(drop_ctr));
  }, py::arg("tables"), py::arg("hdr"), py::arg("state"), py::arg("n"), py::arg("out"), py::arg("out_meta"),
     py::arg("out_state"), py::arg("port_ctr"), py::arg("drop_ctr"));
  m.def("launch_hop_pack", [](uintptr_t out, uintptr_t meta, uintptr_t state, uint32_t n, uintptr_t n_dev,
                              uint32_t plane, uintptr_t fill, uintptr_t count, uintptr_t hdr, uintptr_t dst_state,
                              uintptr_t idx, uint32_t cap, uintptr_t stream) {
    HopInbox d{reinterpret_cast<uint32_t*>(count), reinterpret_cast<uint4*>(hdr), reinterpret_cast<HopState*>(dst_state),
               reinterpret_cast<uint32_t*>(idx), cap};
    check(launch_hop_pack(reinterpret_cast<const void*>(out), reinterpret_cast<const uint32_t*>(meta),
                          reinterpret_cast<const HopState*>(state), n, reinterpret_cast<const uint32_t*>(n_dev), plane,
                          reinterpret_cast<uint32_t*>(fill), d, reinterpret_cast<hipStream_t>(stream)), "launch_hop_pack");
  });
  m.def("launch_resume", [](py::dict tables, uintptr_t count, uintptr_t hdr, uintptr_t state, uintptr_t idx,
                            uint32_t cap, uintptr_t out, uintptr_t out_meta, uintptr_t out_state, uintptr_t port_ctr,
                            uintptr_t drop_ctr, uint32_t flags, int num_cus, uintptr_t stream) {
    const TablesView t = tables_from(tables);
    HopInbox in{reinterpret_cast<uint32_t*>(count), reinterpret_cast<uint4*>(hdr), reinterpret_cast<HopState*>(state),
                reinterpret_cast<uint32_t*>(idx), cap};
    check(launch_resume(t, in, reinterpret_cast<void*>(out), reinterpret_cast<uint32_t*>(out_meta),
                        reinterpret_cast<HopState*>(out_state), reinterpret_cast<unsigned long long*>(port_ctr),
                        reinterpret_cast<unsigned long long*>(drop_ctr), flags, num_cus,
                        reinterpret_cast<hipStream_t>(stream)), "launch_resume");
  });
  // peer access for the hand-off's stores into another GPU's inbox (xGMI); true when the pair can
  // (already enabled counts), false when the devices cannot reach each other
  m.def("enable_peer_access", [](int dev, int peer) -> bool {
    if (dev == peer) return true;
    int can = 0;
    check(hipDeviceCanAccessPeer(&can, dev, peer), "hipDeviceCanAccessPeer");
    if (!can) return false;
    int cur = 0;
    check(hipGetDevice(&cur), "hipGetDevice");
    check(hipSetDevice(dev), "hipSetDevice");
    const hipError_t e = hipDeviceEnablePeerAccess(peer, 0);
    check(hipSetDevice(cur), "hipSetDevice");
    if (e == hipErrorPeerAccessAlreadyEnabled) (void)hipGetLastError();
    else check(e, "hipDeviceEnablePeerAccess");
    return true;
  });
  m.def("mac_learn_cpu", [](uintptr_t macs, uint32_t mask, uintptr_t events, uint32_t n, uint32_t stamp) {
    return mac_learn_cpu(reinterpret_cast<MacEntry*>(macs), mask, reinterpret_cast<const uint32_t*>(events), n, stamp);
  });
  m.def("launch_mac_learn", [](uintptr_t macs, uint32_t mask, uintptr_t events, uintptr_t n_events, uint32_t cap,
                               uint32_t stamp, uintptr_t dropped, uintptr_t stream) {
    check(launch_mac_learn(reinterpret_cast<MacEntry*>(macs), mask, reinterpret_cast<const uint32_t*>(events),
                           reinterpret_cast<const uint32_t*>(n_events), cap, stamp, reinterpret_cast<uint32_t*>(dropped),
                           reinterpret_cast<hipStream_t>(stream)), "mac_learn");
  });

  m.def("fused_lds_bytes", &fused_lds_bytes);
  m.def("launch_fused", [](py::dict tables, uintptr_t pkts, uintptr_t inmeta, uintptr_t out, uintptr_t out_meta,
                           uint32_t n, uintptr_t flow_ctr, uintptr_t port_ctr, uintptr_t drop_ctr, uintptr_t t0,
                           uintptr_t lat, uintptr_t acl_wfrag, uintptr_t acl_cinit, uint32_t acl_tiles,
                           uintptr_t toep_frag, uintptr_t toep_tab, int hash_mode, int acl_mode, int num_cus,
                           uintptr_t stream, uint32_t flags, py::object side, uintptr_t n_dev, uintptr_t steer_list,
                           uintptr_t steer_cnt, uint32_t nranks, uint32_t rank, uint32_t steer_cap,
                           uintptr_t hop_state, uintptr_t v6_keys) {
    FusedLaunch f{};
    f.hop_state = reinterpret_cast<HopState*>(hop_state);
    f.v6_keys = reinterpret_cast<void*>(v6_keys);
    f.steer_list = reinterpret_cast<uint32_t*>(steer_list);
    f.steer_cnt = reinterpret_cast<uint32_t*>(steer_cnt);
    f.steer_cap = steer_cap;
    if (f.steer_list) { f.nranks = nranks; f.rank = rank; }
    f.side = side_from(side);
    f.t = tables_from(tables);
    acl6_from(f, tables);
    f.pkts = reinterpret_cast<const void*>(pkts);
    f.inmeta = reinterpret_cast<const uint32_t*>(inmeta);
    f.out = reinterpret_cast<void*>(out);
    f.out_meta = reinterpret_cast<uint32_t*>(out_meta);
    f.n = n;
    f.flow_ctr = reinterpret_cast<unsigned long long*>(flow_ctr);
    f.port_ctr = reinterpret_cast<unsigned long long*>(port_ctr);
    f.drop_ctr = reinterpret_cast<unsigned long long*>(drop_ctr);
    f.t0 = reinterpret_cast<const unsigned long long*>(t0);
    f.lat = reinterpret_cast<uint32_t*>(lat);
    f.acl_wfrag = reinterpret_cast<const void*>(acl_wfrag);
    f.acl_cinit = reinterpret_cast<const void*>(acl_cinit);
    f.acl_tiles = acl_tiles;
    f.toep_frag = reinterpret_cast<const void*>(toep_frag);
    f.toep_tab = reinterpret_cast<const uint32_t*>(toep_tab);
    f.flags = flags;
    f.n_dev = reinterpret_cast<const uint32_t*>(n_dev);
    if (!f.pkts || !f.inmeta || !f.out || !f.out_meta || !f.port_ctr || !f.drop_ctr)
      throw std::invalid_argument("launch_fused: null buffer");
    if (hash_mode == 2 && !f.toep_frag) throw std::invalid_argument("MFMA hash needs toeplitz frags");
    if (hash_mode == 1 && !f.toep_tab) throw std::invalid_argument("LDS hash needs toeplitz table");
    if (acl_mode == 1 && (!f.acl_wfrag || !f.acl_cinit)) throw std::invalid_argument("MFMA ACL needs frags");
    LaunchCfg cfg;
    cfg.hash_mode = hash_mode; cfg.acl_mode = acl_mode; cfg.num_cus = num_cus;
    check(launch_fused(f, cfg, reinterpret_cast<hipStream_t>(stream)), "launch_fused");
  }, py::arg("tables"), py::arg("pkts"), py::arg("inmeta"), py::arg("out"), py::arg("out_meta"), py::arg("n"),
     py::arg("flow_ctr"), py::arg("port_ctr"), py::arg("drop_ctr"), py::arg("t0"), py::arg("lat"),
     py::arg("acl_wfrag"), py::arg("acl_cinit"), py::arg("acl_tiles"), py::arg("toep_frag"), py::arg("toep_tab"),
     py::arg("hash_mode"), py::arg("acl_mode"), py::arg("num_cus"), py::arg("stream"), py::arg("flags") = 0,
     py::arg("side") = py::none(), py::arg("n_dev") = 0, py::arg("steer_list") = 0, py::arg("steer_cnt") = 0,
     py::arg("nranks") = 0, py::arg("rank") = 0, py::arg("steer_cap") = 0, py::arg("hop_state") = 0,
     py::arg("v6_keys") = 0);
  m.def("launch_pairs", [](py::dict tables, uintptr_t pkts, uintptr_t inmeta, uint32_t n, uintptr_t port_ctr, bool count,
                           uintptr_t stream) {
    const TablesView t = tables_from(tables);
    check(launch_pairs(reinterpret_cast<void*>(pkts), reinterpret_cast<uint32_t*>(inmeta), n, t,
                       reinterpret_cast<unsigned long long*>(port_ctr), count, reinterpret_cast<hipStream_t>(stream)),
          "launch_pairs");
  });
  m.def("launch_pair_fix", [](uintptr_t inmeta, uintptr_t out_meta, uint32_t n, uintptr_t drop_ctr, bool count,
                              uintptr_t stream) {
    check(launch_pair_fix(reinterpret_cast<const uint32_t*>(inmeta), reinterpret_cast<uint32_t*>(out_meta), n,
                          reinterpret_cast<unsigned long long*>(drop_ctr), count, reinterpret_cast<hipStream_t>(stream)),
          "launch_pair_fix");
  });
  m.def("launch_steer", [](uintptr_t pkts, uintptr_t inmeta, uintptr_t list, uintptr_t list_cnt, uint32_t cap_list,
                           uint32_t cnt_len, uintptr_t send, uintptr_t pcnt, uint32_t nranks, uint32_t cap,
                           uintptr_t stream) {
    check(launch_steer(reinterpret_cast<const void*>(pkts), reinterpret_cast<const uint32_t*>(inmeta),
                       reinterpret_cast<const uint32_t*>(list), reinterpret_cast<const uint32_t*>(list_cnt), cap_list,
                       cnt_len, reinterpret_cast<uint8_t*>(send), reinterpret_cast<uint32_t*>(pcnt), nranks, cap,
                       reinterpret_cast<hipStream_t>(stream)), "launch_steer");
  });
  m.def("steer_list_len", &steer_list_len, py::arg("n"), py::arg("num_cus"));
  m.def("gather", [](uintptr_t recv, uint32_t nranks, uint32_t rank, uint32_t cap, uintptr_t pkts, uintptr_t inmeta,
                     uintptr_t n_dev, bool device, uintptr_t stream) -> uint32_t {
    const size_t seg = pkt_seg_bytes(cap), moff = pkt_meta_off(cap);
    if (rank >= nranks || nranks > 64 || seg >= (1ull << 32)) throw std::invalid_argument("gather: bad geometry");
    if (!device) {
      py::gil_scoped_release nogil;
      const uint32_t n = gather_cpu(reinterpret_cast<const uint8_t*>(recv), nranks, rank, cap, (uint32_t)seg,
                                    (uint32_t)moff, reinterpret_cast<uint32_t*>(pkts), reinterpret_cast<uint32_t*>(inmeta));
      if (n_dev) *reinterpret_cast<uint32_t*>(n_dev) = n;
      return n;
    }
    check(launch_gather(reinterpret_cast<const uint8_t*>(recv), nranks, rank, cap, (uint32_t)seg, (uint32_t)moff,
                        reinterpret_cast<void*>(pkts), reinterpret_cast<uint32_t*>(inmeta),
                        reinterpret_cast<uint32_t*>(n_dev), reinterpret_cast<hipStream_t>(stream)), "gather");
    return 0;
  });
  m.def("launch_stamp", [](uintptr_t dst, uintptr_t stream) {
    check(launch_stamp(reinterpret_cast<unsigned long long*>(dst), reinterpret_cast<hipStream_t>(stream)), "stamp");
  });
  m.def("launch_bucket_update", [](uintptr_t idx, uint32_t nb, uintptr_t rows, uintptr_t flows,
                                   uint32_t bucket_mask, uintptr_t stream) {
    check(launch_bucket_update(reinterpret_cast<const uint32_t*>(idx), nb, reinterpret_cast<const void*>(rows),
                               reinterpret_cast<void*>(flows), bucket_mask, reinterpret_cast<hipStream_t>(stream)),
          "bucket_update");
  });
  // ---------------- sharded (multi-GPU) stages: device=True -> HIP kernels, False -> CPU twins
  auto geom = [](const py::dict& d) {
    ShardGeom g;
    g.nranks = val<uint32_t>(d, "nranks", 1); g.rank = val<uint32_t>(d, "rank", 0);
    g.cap_desc = val<uint32_t>(d, "cap_desc", 0); g.cap_pkt = val<uint32_t>(d, "cap_pkt", 0);
    if (g.rank >= g.nranks || g.nranks > 127 || g.cap_desc >= (1u << 24)) throw std::invalid_argument("bad shard geometry");
    return g;
  };
  m.def("desc_seg_bytes", [](uint32_t cap) { return desc_seg_bytes(cap); });
  m.def("verdict_seg_bytes", [](uint32_t cap) { return verdict_seg_bytes(cap); });
  m.def("pkt_seg_bytes", [](uint32_t cap) { return pkt_seg_bytes(cap); });
  m.def("pkt_meta_off", [](uint32_t cap) { return pkt_meta_off(cap); });
  m.def("shard_ingress", [geom](py::dict tables, py::dict d, bool device, int hash_mode, int acl_mode, int num_cus,
                                uintptr_t stream) {
    IngressArgs a{};
    a.t = tables_from(tables);
    a.t.flow6_on = 0;   // IPv6 flows need the addresses at the probe: not on the sharded path (shard.hip)
    a.pkts = ptr<const uint4>(d, "pkts"); a.inmeta = ptr<const uint32_t>(d, "inmeta");
    a.n = val<uint32_t>(d, "n", 0); a.g = geom(d);
    a.send_desc = ptr<uint8_t>(d, "send_desc"); a.cnt = ptr<uint32_t>(d, "cnt");
    a.ref = ptr<uint32_t>(d, "ref"); a.aux = ptr<uint32_t>(d, "aux");
    a.acl_wfrag = ptr<const void>(d, "acl_wfrag"); a.acl_cinit = ptr<const void>(d, "acl_cinit");
    a.acl_tiles = val<uint32_t>(d, "acl_tiles", 1);
    a.toep_frag = ptr<const void>(d, "toep_frag"); a.toep_tab = ptr<const uint32_t>(d, "toep_tab");
    if (!a.pkts || !a.inmeta || !a.send_desc || !a.cnt || !a.ref || !a.aux) throw std::invalid_argument("ingress: null buffer");
    if (!device) { py::gil_scoped_release nogil; ingress_cpu(a); return; }
    if (hash_mode == 2 && !a.toep_frag) throw std::invalid_argument("MFMA hash needs toeplitz frags");
    if (!a.toep_tab) throw std::invalid_argument("ingress needs the toeplitz table");
    if (acl_mode == 1 && (!a.acl_wfrag || !a.acl_cinit)) throw std::invalid_argument("MFMA ACL needs frags");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    check(launch_ingress(a, hash_mode, acl_mode, num_cus, s), "shard_ingress");
    check(launch_seg_headers(a.cnt, a.send_desc, a.g.nranks, desc_seg_bytes(a.g.cap_desc), a.g.cap_desc, s), "seg_headers");
  });
  m.def("shard_owner", [geom](py::dict tables, py::dict d, bool device, int num_cus, uintptr_t stream) {
    OwnerArgs a{};
    a.t = tables_from(tables); a.g = geom(d);
    a.recv_desc = ptr<const uint8_t>(d, "recv_desc"); a.send_verdict = ptr<uint8_t>(d, "send_verdict");
    a.flow_ctr = ptr<unsigned long long>(d, "flow_ctr"); a.toep_tab = ptr<const uint32_t>(d, "toep_tab");
    if (!a.recv_desc || !a.send_verdict) throw std::invalid_argument("owner: null buffer");
    if (!device) { py::gil_scoped_release nogil; owner_cpu(a); return; }
    if (!a.toep_tab) throw std::invalid_argument("owner needs the toeplitz table");
    check(launch_owner(a, num_cus, reinterpret_cast<hipStream_t>(stream)), "shard_owner");
  });
  m.def("shard_apply", [geom](py::dict tables, py::dict d, bool device, int num_cus, uintptr_t stream) {
    ApplyArgs a{};
    a.t = tables_from(tables); a.g = geom(d);
    a.pkts = ptr<const uint4>(d, "pkts"); a.inmeta = ptr<const uint32_t>(d, "inmeta"); a.n = val<uint32_t>(d, "n", 0);
    a.ref = ptr<const uint32_t>(d, "ref"); a.aux = ptr<const uint32_t>(d, "aux");
    a.recv_verdict = ptr<const uint8_t>(d, "recv_verdict"); a.out = ptr<uint4>(d, "out");
    a.out_meta = ptr<uint32_t>(d, "out_meta"); a.send_pkt = ptr<uint8_t>(d, "send_pkt"); a.pcnt = ptr<uint32_t>(d, "pcnt");
    a.port_ctr = ptr<unsigned long long>(d, "port_ctr"); a.drop_ctr = ptr<unsigned long long>(d, "drop_ctr");
    a.t0 = ptr<const unsigned long long>(d, "t0"); a.lat = ptr<uint32_t>(d, "lat");
    if (!a.pkts || !a.inmeta || !a.ref || !a.aux || !a.recv_verdict || !a.out || !a.out_meta || !a.send_pkt || !a.pcnt ||
        !a.port_ctr || !a.drop_ctr)
      throw std::invalid_argument("apply: null buffer");
    if (!device) { py::gil_scoped_release nogil; apply_cpu(a); return; }
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    check(launch_apply(a, num_cus, s), "shard_apply");
    check(launch_seg_headers(a.pcnt, a.send_pkt, a.g.nranks, pkt_seg_bytes(a.g.cap_pkt), a.g.cap_pkt, s), "seg_headers");
  });
  m.def("shard_egress", [geom](py::dict d, bool device, int num_cus, uintptr_t stream) {
    EgressArgs a{};
    a.g = geom(d);
    a.recv_pkt = ptr<const uint8_t>(d, "recv_pkt"); a.port_ctr = ptr<unsigned long long>(d, "port_ctr");
    a.t0 = ptr<const unsigned long long>(d, "t0"); a.lat = ptr<uint32_t>(d, "lat");
    if (!a.recv_pkt || !a.port_ctr) throw std::invalid_argument("egress: null buffer");
    if (!device) { py::gil_scoped_release nogil; egress_cpu(a); return; }
    check(launch_egress(a, num_cus, reinterpret_cast<hipStream_t>(stream)), "shard_egress");
  });

  // Replicated-table multi-GPU step: fused kernel with per-GPU egress segments (device=True) or
  // its CPU twin (device=False).  d: tables-independent buffers + geometry (nranks, rank, cap_pkt).
  m.def("fused_remote", [geom](py::dict tables, py::dict d, bool device, int hash_mode, int acl_mode, int num_cus,
                               uintptr_t stream) {
    ShardGeom g = geom(d);
    FusedLaunch f{};
    f.t = tables_from(tables);
    acl6_from(f, tables);
    f.pkts = ptr<const void>(d, "pkts"); f.inmeta = ptr<const uint32_t>(d, "inmeta");
    f.out = ptr<void>(d, "out"); f.out_meta = ptr<uint32_t>(d, "out_meta"); f.n = val<uint32_t>(d, "n", 0);
    f.flow_ctr = ptr<unsigned long long>(d, "flow_ctr"); f.port_ctr = ptr<unsigned long long>(d, "port_ctr");
    f.drop_ctr = ptr<unsigned long long>(d, "drop_ctr");
    f.t0 = ptr<const unsigned long long>(d, "t0"); f.lat = ptr<uint32_t>(d, "lat");
    f.acl_wfrag = ptr<const void>(d, "acl_wfrag"); f.acl_cinit = ptr<const void>(d, "acl_cinit");
    f.acl_tiles = val<uint32_t>(d, "acl_tiles", 1);
    f.toep_frag = ptr<const void>(d, "toep_frag"); f.toep_tab = ptr<const uint32_t>(d, "toep_tab");
    f.flags = val<uint32_t>(d, "flags", 0);
    f.send_pkt = ptr<uint8_t>(d, "send_pkt"); f.pcnt = ptr<uint32_t>(d, "pcnt");
    f.nranks = g.nranks; f.rank = g.rank; f.cap_pkt = g.cap_pkt;
    f.steer = val<uint32_t>(d, "steer", 0);
    if (!f.pkts || !f.inmeta || !f.out || !f.out_meta || !f.port_ctr || !f.drop_ctr || !f.send_pkt || !f.pcnt)
      throw std::invalid_argument("fused_remote: null buffer");
    if (g.nranks < 2) throw std::invalid_argument("fused_remote needs nranks >= 2");
    if (!device) {
      RemoteOut r{g.nranks, g.rank, g.cap_pkt, f.send_pkt, f.pcnt, f.steer};
      py::gil_scoped_release nogil;
      oracle_run_remote(f.t, reinterpret_cast<const uint32_t*>(f.pkts), f.inmeta, f.n,
                        reinterpret_cast<uint32_t*>(f.out), f.out_meta, reinterpret_cast<uint64_t*>(f.flow_ctr),
                        reinterpret_cast<uint64_t*>(f.port_ctr), reinterpret_cast<uint64_t*>(f.drop_ctr), r);
      return;
    }
    if (hash_mode == 2 && !f.toep_frag) throw std::invalid_argument("MFMA hash needs toeplitz frags");
    if (hash_mode == 1 && !f.toep_tab) throw std::invalid_argument("LDS hash needs toeplitz table");
    if (acl_mode == 1 && (!f.acl_wfrag || !f.acl_cinit)) throw std::invalid_argument("MFMA ACL needs frags");
    LaunchCfg cfg;
    cfg.hash_mode = hash_mode; cfg.acl_mode = acl_mode; cfg.num_cus = num_cus;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    check(launch_fused(f, cfg, s), "fused_remote");
    check(launch_seg_headers(f.pcnt, f.send_pkt, g.nranks, pkt_seg_bytes(g.cap_pkt), g.cap_pkt, s), "seg_headers");
  });

  // Host <-> HBM packet I/O engine (pinned host slots, SDMA streams, event-chained kernel).
  py::class_<PacketIo>(m, "PacketIo")
      .def(py::init<uint32_t, uint32_t>(), py::arg("capacity"), py::arg("depth") = 3)
      .def_property_readonly("capacity", &PacketIo::capacity)
      .def_property_readonly("depth", &PacketIo::depth)
      .def("host_in", [](py::object self, uint32_t s) {
        PacketIo& io = self.cast<PacketIo&>();
        if (s >= io.depth()) throw std::out_of_range("slot");
        return py::array_t<uint8_t>({(py::ssize_t)io.capacity(), (py::ssize_t)64}, io.host_in(s), self);
      })
      .def("host_inmeta", [](py::object self, uint32_t s) {
        PacketIo& io = self.cast<PacketIo&>();
        if (s >= io.depth()) throw std::out_of_range("slot");
        return py::array_t<uint32_t>({(py::ssize_t)io.capacity()}, io.host_inmeta(s), self);
      })
      .def("host_out", [](py::object self, uint32_t s) {
        PacketIo& io = self.cast<PacketIo&>();
        if (s >= io.depth()) throw std::out_of_range("slot");
        return py::array_t<uint8_t>({(py::ssize_t)io.capacity(), (py::ssize_t)64}, io.host_out(s), self);
      })
      .def("host_meta", [](py::object self, uint32_t s) {
        PacketIo& io = self.cast<PacketIo&>();
        if (s >= io.depth()) throw std::out_of_range("slot");
        return py::array_t<uint32_t>({(py::ssize_t)io.capacity()}, io.host_meta(s), self);
      })
      .def("dev_lat", [](PacketIo& io, uint32_t s) { return reinterpret_cast<uintptr_t>(io.dev_lat(s)); })
      .def("submit", [](PacketIo& io, uint32_t s, uint32_t n, py::dict tables, py::dict d, int hash_mode, int acl_mode,
                        int num_cus) {
        FusedLaunch f{};
        f.t = tables_from(tables);
        acl6_from(f, tables);
        f.flow_ctr = ptr<unsigned long long>(d, "flow_ctr"); f.port_ctr = ptr<unsigned long long>(d, "port_ctr");
        f.drop_ctr = ptr<unsigned long long>(d, "drop_ctr"); f.t0 = ptr<const unsigned long long>(d, "t0");
        f.acl_wfrag = ptr<const void>(d, "acl_wfrag"); f.acl_cinit = ptr<const void>(d, "acl_cinit");
        f.acl_tiles = val<uint32_t>(d, "acl_tiles", 1);
        f.toep_frag = ptr<const void>(d, "toep_frag"); f.toep_tab = ptr<const uint32_t>(d, "toep_tab");
        f.flags = val<uint32_t>(d, "flags", 0);
        if (!f.flow_ctr || !f.port_ctr || !f.drop_ctr) throw std::invalid_argument("pktio submit: null counters");
        if (hash_mode == 2 && !f.toep_frag) throw std::invalid_argument("MFMA hash needs toeplitz frags");
        if (hash_mode == 1 && !f.toep_tab) throw std::invalid_argument("LDS hash needs toeplitz table");
        if (acl_mode == 1 && (!f.acl_wfrag || !f.acl_cinit)) throw std::invalid_argument("MFMA ACL needs frags");
        LaunchCfg cfg;
        cfg.hash_mode = hash_mode; cfg.acl_mode = acl_mode; cfg.num_cus = num_cus;
        io.submit(s, n, f, cfg);
      })
      .def("wait", [](PacketIo& io, uint32_t s) { py::gil_scoped_release nogil; io.wait(s); })
      .def("ready", &PacketIo::ready)
      .def("timings", [](PacketIo& io, uint32_t s) {
        float a, b, c, t;
        io.timings(s, &a, &b, &c, &t);
        return py::make_tuple(a, b, c, t);
      });

  // Blocking copy between any two addresses (device or host; unified addressing).
  // Copy on a private non-blocking stream: never ordered behind a resident (ring) kernel.
  m.def("memcpy_nb", [](uintptr_t dst, uintptr_t src, size_t nbytes) {
    py::gil_scoped_release nogil;
    static hipStream_t s = [] {
      hipStream_t x{};
      check(hipStreamCreateWithFlags(&x, hipStreamNonBlocking), "stream");
      return x;
    }();
    check(hipMemcpyAsync(reinterpret_cast<void*>(dst), reinterpret_cast<const void*>(src), nbytes, hipMemcpyDefault, s),
          "memcpy_nb");
    check(hipStreamSynchronize(s), "memcpy_nb");
  });
  m.def("memcpy", [](uintptr_t dst, uintptr_t src, size_t nbytes) {
    py::gil_scoped_release nogil;
    check(hipMemcpy(reinterpret_cast<void*>(dst), reinterpret_cast<const void*>(src), nbytes, hipMemcpyDefault),
          "memcpy");
  });

  // Persistent ring kernel (low-latency path): the host publishes 64-packet chunks, resident
  // waves process them as they appear, completion flags come back through pinned host memory.
  py::class_<RingEngine>(m, "RingEngine")
      .def(py::init<uint32_t, int, int, bool, bool, uint32_t>(), py::arg("capacity"), py::arg("num_cus"),
           py::arg("wgs_per_cu") = 1, py::arg("coop") = true, py::arg("host_slots") = false, py::arg("queues") = 1)
      .def_property_readonly("queues", &RingEngine::queues)
      .def_property_readonly("host_slots", &RingEngine::host_slots)
      .def_property_readonly("capacity", &RingEngine::capacity)
      .def_property_readonly("running", &RingEngine::running)
      .def("alive", &RingEngine::alive)
      .def_property_readonly("published", [](const RingEngine& r) { return r.published(0); })
      .def("published_q", &RingEngine::published, py::arg("q") = 0)
      .def("dev_in", [](RingEngine& r) { return reinterpret_cast<uintptr_t>(r.dev_in()); })
      .def("dev_inmeta", [](RingEngine& r) { return reinterpret_cast<uintptr_t>(r.dev_inmeta()); })
      .def("dev_out", [](RingEngine& r) { return reinterpret_cast<uintptr_t>(r.dev_out()); })
      .def("dev_meta", [](RingEngine& r) { return reinterpret_cast<uintptr_t>(r.dev_meta()); })
      .def("dev_svc", [](RingEngine& r) { return reinterpret_cast<uintptr_t>(r.dev_svc()); })
      .def("host_view", [](RingEngine& r) {
        // host addresses of the pinned slot buffers (host_slots rings): in, inmeta, out, meta
        if (!r.host_slots()) throw std::runtime_error("ring: host_view needs host_slots=True");
        return py::make_tuple(reinterpret_cast<uintptr_t>(r.host_ptr(0)), reinterpret_cast<uintptr_t>(r.host_ptr(1)),
                              reinterpret_cast<uintptr_t>(r.host_ptr(2)), reinterpret_cast<uintptr_t>(r.host_ptr(3)));
      })
      .def("start", [](RingEngine& r, py::dict tables, py::dict d, int hash_mode, int acl_mode, int num_cus,
                       double deadline_s) {
        FusedLaunch f{};
        f.t = tables_from(tables);
        acl6_from(f, tables);
        f.flow_ctr = ptr<unsigned long long>(d, "flow_ctr"); f.port_ctr = ptr<unsigned long long>(d, "port_ctr");
        f.drop_ctr = ptr<unsigned long long>(d, "drop_ctr");
        f.acl_wfrag = ptr<const void>(d, "acl_wfrag"); f.acl_cinit = ptr<const void>(d, "acl_cinit");
        f.acl_tiles = val<uint32_t>(d, "acl_tiles", 1);
        f.toep_frag = ptr<const void>(d, "toep_frag"); f.toep_tab = ptr<const uint32_t>(d, "toep_tab");
        f.flags = val<uint32_t>(d, "flags", 0);
        if (d.contains("side")) f.side = side_from(d["side"]);
        f.side.blk_cnt = nullptr;   // the ring appends to one flat list
        if (f.side.cnt && (!f.side.list || f.side.cap_list < r.capacity()))
          throw std::invalid_argument("ring side list must hold a whole ring");
        if (!f.port_ctr || !f.drop_ctr) throw std::invalid_argument("ring start: null counters");
        if (hash_mode == 2 && !f.toep_frag) throw std::invalid_argument("MFMA hash needs toeplitz frags");
        if (hash_mode == 1 && !f.toep_tab) throw std::invalid_argument("LDS hash needs toeplitz table");
        if (acl_mode == 1 && (!f.acl_wfrag || !f.acl_cinit)) throw std::invalid_argument("MFMA ACL needs frags");
        LaunchCfg cfg;
        cfg.hash_mode = hash_mode; cfg.acl_mode = acl_mode; cfg.num_cus = num_cus;
        r.start(f, cfg, deadline_s, ptr<const void>(tables, "flows_alt"));
      })
      .def("stage_tables", [](RingEngine& r, py::dict tables, py::dict d, int which) {
        FusedLaunch f{};
        f.t = tables_from(tables);
        acl6_from(f, tables);
        f.acl_wfrag = ptr<const void>(d, "acl_wfrag"); f.acl_cinit = ptr<const void>(d, "acl_cinit");
        f.acl_tiles = val<uint32_t>(d, "acl_tiles", 1);
        f.toep_frag = ptr<const void>(d, "toep_frag"); f.toep_tab = ptr<const uint32_t>(d, "toep_tab");
        py::gil_scoped_release nogil;
        r.stage_tables(f, which);
      })
      .def("flip_tables", &RingEngine::flip_tables)
      .def_property_readonly("table_set", &RingEngine::table_set)
      .def_property_readonly("lds_acl_tiles", &RingEngine::lds_acl_tiles)
      .def("flip", &RingEngine::flip)
      .def("change_epoch", &RingEngine::change_epoch, py::arg("flow"), py::arg("set"))
      // control mailbox: dwords to a device address, applied by the running grid
      .def("post_write", [](RingEngine& r, uint64_t dst, py::bytes data, double timeout_s) {
        std::string s = data;
        if (s.size() % 4) throw std::invalid_argument("ring: control data is whole dwords");
        std::vector<uint32_t> w(s.size() / 4);
        std::memcpy(w.data(), s.data(), s.size());
        py::gil_scoped_release nogil;
        return r.post_write(dst, w.data(), (uint32_t)w.size(), timeout_s);
      }, py::arg("dst"), py::arg("data"), py::arg("timeout_s") = 1.0)
      .def_property_readonly("ctrl_done", &RingEngine::ctrl_done)
      // GPU-direct egress (ring.h GdeRing)
      .def("gde_enable", &RingEngine::gde_enable, py::arg("on") = true)
      .def_property_readonly("gde_on", &RingEngine::gde_on)
      .def("gde_set", &RingEngine::gde_set, py::arg("port"), py::arg("q"), py::arg("ctl"), py::arg("desc"), py::arg("buf"),
           py::arg("ring_size"), py::arg("buf_size"), py::arg("head") = 0, py::arg("tail") = 0,
           py::call_guard<py::gil_scoped_release>())
      .def("gde_clear", &RingEngine::gde_clear, py::arg("port"), py::arg("q"), py::call_guard<py::gil_scoped_release>())
      .def("gde_stats", &RingEngine::gde_stats)
      // SFC hops across GPUs in the live path (ring.h XferEntry)
      .def("xfer_enable", &RingEngine::xfer_enable, py::arg("entries"), py::arg("wgs") = 1)
      .def_property_readonly("xfer_on", &RingEngine::xfer_on)
      .def_property_readonly("xfer_active", &RingEngine::xfer_active)
      .def("xfer_desc", [](const RingEngine& r) {
        const RingEngine::XferDesc d = r.xfer_desc();
        py::dict o;
        o["inbox"] = d.inbox; o["entries"] = d.entries; o["out"] = d.out; o["out_meta"] = d.out_meta;
        o["xpend"] = d.xpend; o["cap"] = d.cap; o["ring_mask"] = d.ring_mask; o["nq"] = d.nq;
        return o;
      })
      .def("xfer_set_peers", [](RingEngine& r, uint32_t my_plane, py::list planes) {
        std::vector<RingEngine::XferDesc> v;
        for (auto o : planes) {
          py::dict d = o.cast<py::dict>();
          RingEngine::XferDesc x;
          x.inbox = d["inbox"].cast<uint64_t>(); x.entries = d["entries"].cast<uint64_t>();
          x.out = d["out"].cast<uint64_t>(); x.out_meta = d["out_meta"].cast<uint64_t>();
          x.xpend = d["xpend"].cast<uint64_t>(); x.cap = d["cap"].cast<uint32_t>();
          x.ring_mask = d["ring_mask"].cast<uint32_t>(); x.nq = d["nq"].cast<uint32_t>();
          v.push_back(x);
        }
        r.xfer_set_peers(my_plane, v);
      }, py::arg("my_plane"), py::arg("planes"))
      .def("xfer_stats", &RingEngine::xfer_stats)
      .def_property_readonly("ctrl_posted", &RingEngine::ctrl_posted)
      .def("wait_ctrl", [](RingEngine& r, uint64_t seq, double timeout_s) {
        py::gil_scoped_release nogil;
        return r.wait_ctrl(seq, timeout_s);
      }, py::arg("seq"), py::arg("timeout_s") = 1.0)
      .def("set_ctrl_regions", &RingEngine::set_ctrl_regions)
      .def("bump_epoch", &RingEngine::bump_epoch)
      .def("grace_over", &RingEngine::grace_over)
      .def("wait_grace", [](RingEngine& r, double timeout_s) {
        py::gil_scoped_release nogil;
        return r.wait_grace(timeout_s);
      }, py::arg("timeout_s") = 10.0)
      .def_property_readonly("epoch", &RingEngine::epoch)
      .def("set_epoch", &RingEngine::set_epoch)
      .def("set_frame_addrs", &RingEngine::set_frame_addrs, py::arg("on"))
      .def_property_readonly("frame_addrs_on", &RingEngine::frame_addrs_on)
      .def("stop", [](RingEngine& r, double timeout_s) { py::gil_scoped_release nogil; r.stop(timeout_s); },
           py::arg("timeout_s") = 30.0)
      .def("completed", &RingEngine::completed, py::arg("q") = 0)
      .def("publish", &RingEngine::publish, py::arg("n"), py::arg("check_room") = true, py::arg("q") = 0)
      .def("wait", [](RingEngine& r, uint64_t end, double timeout_s, uint32_t q) {
        py::gil_scoped_release nogil;
        return r.wait(end, timeout_s, q);
      }, py::arg("end"), py::arg("timeout_s") = 10.0, py::arg("q") = 0)
      .def("probe", [](RingEngine& r, uint32_t batches, uint32_t batch, uint32_t inflight) {
        double el = 0;
        std::vector<double> v;
        {
          py::gil_scoped_release nogil;
          v = r.probe(batches, batch, inflight, &el);
        }
        return py::make_tuple(py::array_t<double>(v.size(), v.data()), el);
      });

  m.def("launch_side", [](py::dict tables, uintptr_t pkts, uintptr_t inmeta, uintptr_t out, uintptr_t out_meta,
                          py::object side, uintptr_t port_ctr, uintptr_t drop_ctr, uintptr_t stream, uint32_t n_slots,
                          bool wrap) {
    const TablesView t = tables_from(tables);
    SideOut so = side_from(side);
    so.blk_cnt = nullptr;       // standalone side pass / oracle: one flat list
    check(launch_side(t, reinterpret_cast<const void*>(pkts), reinterpret_cast<const uint32_t*>(inmeta),
                      reinterpret_cast<const void*>(out), reinterpret_cast<const uint32_t*>(out_meta), so,
                      reinterpret_cast<unsigned long long*>(port_ctr), reinterpret_cast<unsigned long long*>(drop_ctr),
                      reinterpret_cast<hipStream_t>(stream), n_slots, wrap), "launch_side");
  }, py::arg("tables"), py::arg("pkts"), py::arg("inmeta"), py::arg("out"), py::arg("out_meta"), py::arg("side"),
     py::arg("port_ctr"), py::arg("drop_ctr"), py::arg("stream"), py::arg("n_slots") = 0, py::arg("wrap") = false);
  // ---- IPsec ESP engine ----
  m.attr("ESP_SA_BYTES") = (int)sizeof(EspSa);
  m.attr("ESP_CLEAR_OFF") = kClearOff;
  m.attr("ESP_OFF") = kEspOff;
  m.def("esp_tables", []() {
    const EspTables t = esp_host_tables();
    return py::make_tuple(py::bytes(reinterpret_cast<const char*>(t.te0), 4096),
                          py::bytes(reinterpret_cast<const char*>(t.sbox), 256),
                          py::bytes(reinterpret_cast<const char*>(t.rem), 2048));
  });
  m.def("esp_build_sa", [](py::bytes key, py::bytes salt, uint32_t spi, uint32_t mode, uint32_t src_raw,
                           uint32_t dst_raw, uint32_t smac_lo, uint32_t smac_hi, uint32_t dmac_lo, uint32_t dmac_hi) {
    std::string k = key, sl = salt;
    if (sl.size() != 4) throw std::invalid_argument("ESP: salt must be 4 bytes");
    const EspSa sa = esp_build_sa(reinterpret_cast<const uint8_t*>(k.data()), k.size(),
                                  reinterpret_cast<const uint8_t*>(sl.data()), spi, mode, src_raw, dst_raw, smac_lo,
                                  (uint16_t)smac_hi, dmac_lo, (uint16_t)dmac_hi);
    return py::bytes(reinterpret_cast<const char*>(&sa), sizeof(sa));
  });
  m.def("esp_run_cpu", [](bool enc, py::dict d) { esp_run_cpu(esp_from(d), enc); });
  m.def("launch_esp", [](bool enc, py::dict d, uintptr_t te0, uintptr_t sbox, uintptr_t rem, int num_cus,
                         uintptr_t stream) {
    check(launch_esp(esp_from(d), enc, reinterpret_cast<const uint32_t*>(te0), reinterpret_cast<const uint8_t*>(sbox),
                     reinterpret_cast<const uint64_t*>(rem), num_cus, reinterpret_cast<hipStream_t>(stream)),
          "launch_esp");
  });
  m.def("launch_harvest", [](uintptr_t ctr, uintptr_t out, uint32_t n, uintptr_t stream) {
    check(launch_harvest(reinterpret_cast<unsigned long long*>(ctr), reinterpret_cast<unsigned long long*>(out), n,
                         reinterpret_cast<hipStream_t>(stream)), "harvest");
  });

  // ---- native packet I/O engine (iox.h): ports, backends, engine; pod-side memif tools ----
  using namespace nfdp::iox;
  py::class_<Port, std::shared_ptr<Port>>(m, "IoPort")
      .def_property_readonly("kind", &Port::kind)
      .def("counters", [](Port& p) {
        return py::dict(py::arg("rx") = p.rx_pkts.load(), py::arg("tx") = p.tx_pkts.load(),
                        py::arg("tx_full") = p.tx_full.load(), py::arg("rx_bytes") = p.rx_bytes.load(),
                        py::arg("tx_bytes") = p.tx_bytes.load());
      });
  py::class_<MemifPort, Port, std::shared_ptr<MemifPort>>(m, "MemifPort")
      .def(py::init<const std::string&, uint32_t, uint32_t, uint32_t>(), py::arg("path"), py::arg("ring_size") = 1024,
           py::arg("buf_size") = 2048, py::arg("tx_rings") = 1)
      .def_property_readonly("tx_rings", &MemifPort::tx_queues)
      .def_property_readonly("path", &MemifPort::path);
  py::class_<PacketPort, Port, std::shared_ptr<PacketPort>>(m, "PacketPort")
      .def(py::init<const std::string&, uint32_t, uint32_t>(), py::arg("ifname"), py::arg("frames") = 1024,
           py::arg("frame_size") = 2048);
  py::class_<XdpPort, Port, std::shared_ptr<XdpPort>>(m, "XdpPort")
      .def(py::init<const std::string&, uint32_t, uint32_t, uint32_t>(), py::arg("ifname"), py::arg("frames") = 2048,
           py::arg("frame_size") = 2048, py::arg("queue") = 0)
      .def_property_readonly("native_mode", &XdpPort::native_mode);
  py::class_<FdPort, Port, std::shared_ptr<FdPort>>(m, "FdPort")
      .def(py::init<int, uint32_t, uint32_t>(), py::arg("fd"), py::arg("nbufs") = 256, py::arg("buf_size") = 9728);
  py::class_<Backend, std::shared_ptr<Backend>>(m, "IoBackend")
      .def_property_readonly("capacity", &Backend::capacity)
      .def_property_readonly("queues", &Backend::queues)
      .def("published", &Backend::published, py::arg("q") = 0);
  py::class_<GpuBackend, Backend, std::shared_ptr<GpuBackend>>(m, "GpuBackend")
      .def(py::init<RingEngine*>(), py::arg("ring"), py::keep_alive<1, 2>());
  py::class_<OracleBackend, Backend, std::shared_ptr<OracleBackend>>(m, "OracleBackend")
      .def(py::init<uint32_t, uint32_t>(), py::arg("capacity"), py::arg("queues") = 1)
      .def("configure", [](OracleBackend& b, py::dict tables, uintptr_t flow_ctr, uintptr_t port_ctr, uintptr_t drop_ctr) {
        const TablesView t = tables_from(tables);
        b.configure(t, reinterpret_cast<uint64_t*>(flow_ctr), reinterpret_cast<uint64_t*>(port_ctr),
                    reinterpret_cast<uint64_t*>(drop_ctr), const_cast<MacEntry*>(t.macs), t.mac_mask);
      })
      .def("set_frame_addrs", &OracleBackend::set_frame_addrs, py::arg("on"))
      .def("set_completion_gate", &OracleBackend::set_completion_gate, py::arg("on"));
  py::class_<WireBackend, OracleBackend, std::shared_ptr<WireBackend>>(m, "WireBackend")
      .def(py::init<uint32_t, uint32_t, const std::vector<std::pair<uint64_t, uint32_t>>&>(), py::arg("capacity"),
           py::arg("queues"), py::arg("mac_to_port"));
  // host snapshot of the side pass's tables: host arrays (numpy) copied at construction
  py::class_<SideTables, std::shared_ptr<SideTables>>(m, "SideTables")
      .def(py::init([](py::buffer ports, py::buffer macs, uint32_t mac_mask, py::buffer lag, uint32_t n_lag_groups,
                       py::buffer flood, uint32_t n_flood, py::buffer tunnels, uint32_t n_tunnels, py::buffer tunnels6,
                       uint32_t n_tunnels6, py::bytes rss, bool v6) {
        auto req = [](py::buffer& b, size_t elem, size_t need, const char* what) {
          py::buffer_info bi = b.request();
          const size_t bytes = (size_t)bi.size * bi.itemsize;
          if (bytes < need * elem) throw std::invalid_argument(std::string("SideTables: ") + what + " too small");
          return std::make_pair(bi.ptr, bytes / elem);
        };
        SideTables::Src src{};
        auto pp = req(ports, sizeof(PortEntry), 1, "ports");
        src.ports = static_cast<const PortEntry*>(pp.first); src.n_ports = pp.second;
        auto mp = req(macs, sizeof(MacEntry), (size_t)mac_mask + 1, "macs");
        src.macs = static_cast<const MacEntry*>(mp.first); src.mac_mask = mac_mask;
        auto lp = req(lag, 2, (size_t)n_lag_groups * kLagWays, "lag");
        src.lag = static_cast<const uint16_t*>(lp.first); src.n_lag_groups = n_lag_groups;
        auto fp = req(flood, 2, (size_t)n_flood * kFloodWays, "flood");
        src.flood = static_cast<const uint16_t*>(fp.first); src.flood_rows = fp.second / kFloodWays; src.n_flood = n_flood;
        if (src.flood_rows > kFloodMaxRows) throw std::invalid_argument("SideTables: flood rows beyond kFloodMaxRows");
        auto tp = req(tunnels, sizeof(TunnelEntry), n_tunnels, "tunnels");
        src.tunnels = static_cast<const TunnelEntry*>(tp.first); src.n_tunnels = n_tunnels;
        auto t6 = req(tunnels6, sizeof(Tunnel6Entry), n_tunnels6, "tunnels6");
        src.tunnels6 = static_cast<const Tunnel6Entry*>(t6.first); src.n_tunnels6 = n_tunnels6;
        std::string k = rss;
        if (k.size() < 52) k.resize(52, '\0');
        src.rss_key = reinterpret_cast<const uint8_t*>(k.data());
        src.v6 = v6;
        return std::make_shared<SideTables>(src);
      }), py::arg("ports"), py::arg("macs"), py::arg("mac_mask"), py::arg("lag"), py::arg("n_lag_groups"),
         py::arg("flood"), py::arg("n_flood"), py::arg("tunnels"), py::arg("n_tunnels"), py::arg("tunnels6"),
         py::arg("n_tunnels6"), py::arg("rss"), py::arg("v6") = false)
      .def("mac_lookup", [](SideTables& t, uint32_t bridge, uint32_t lo, uint32_t hi) {
        std::shared_lock<std::shared_mutex> g(t.mac_mu);
        return mac_lookup(t.view(), bridge, lo, hi);
      });
  py::class_<Engine>(m, "IoEngine")
      .def(py::init<uint32_t, uint32_t, uint32_t, uint32_t, uint32_t>(), py::arg("burst") = 256,
           py::arg("inflight") = 64, py::arg("tx_workers") = 1, py::arg("queues") = 1,
           py::arg("max_inflight_frames") = 0)
      .def_property_readonly("queues", &Engine::queues)
      .def("add_backend", &Engine::add_backend)
      .def("add_port", &Engine::add_port, py::arg("id"), py::arg("port"), py::arg("queue") = -1)
      .def("remove_port", &Engine::remove_port)
      .def("retired_ports", &Engine::retired_ports, py::call_guard<py::gil_scoped_release>())
      .def("port", &Engine::port)
      .def("port_queue", &Engine::port_queue)
      .def("set_side_tables", &Engine::set_side_tables)
      .def("set_redirects", &Engine::set_redirects)
      .def("set_coalesce", &Engine::set_coalesce, py::arg("frames") = 64, py::arg("window_us") = 0.0)
      .def("set_queue_cpus", &Engine::set_queue_cpus, py::arg("queue"), py::arg("cpus"))
      .def("set_zero_copy", &Engine::set_zero_copy, py::arg("on"))
      .def("set_gpu_egress", &Engine::set_gpu_egress, py::arg("on"))
      .def_property_readonly("gpu_egress", &Engine::gpu_egress)
      .def_property_readonly("zero_copy", &Engine::zero_copy)
      .def("hold", [](Engine& e) { py::gil_scoped_release nogil; e.hold(); })
      .def("release", &Engine::release)
      .def("flush_learning", [](Engine& e) { py::gil_scoped_release nogil; e.flush_learning(); })
      .def_property("learn_stamp", &Engine::learn_stamp, &Engine::set_learn_stamp)
      .def("side_port_counters", [](const Engine& e) {
        auto v = e.side_port_counters();
        return py::array_t<uint64_t>(v.size(), v.data());
      })
      .def("side_drop_counters", [](const Engine& e) {
        auto v = e.side_drop_counters();
        return py::array_t<uint64_t>(v.size(), v.data());
      })
      .def("set_steering", [](Engine& e, py::buffer ports, py::bytes rss, bool v6, std::vector<uint32_t> port_owner) {
        py::buffer_info bi = ports.request();
        const size_t n = (size_t)bi.size * bi.itemsize / sizeof(PortEntry);
        std::vector<PortEntry> v(n);
        std::memcpy(v.data(), bi.ptr, n * sizeof(PortEntry));
        std::string k = rss;
        e.set_steering(v, std::vector<uint8_t>(k.begin(), k.end()), v6, port_owner);
      }, py::arg("ports"), py::arg("rss"), py::arg("v6") = false, py::arg("port_owner") = std::vector<uint32_t>{})
      .def("set_redirect", &Engine::set_redirect)
      .def("set_side_ports", &Engine::set_side_ports)
      // A live commit's switch in one native call, without the GIL: hold publication (every rx
      // thread between two bursts), change every ring's epoch (flow copy and / or table set), swap
      // in the side-table snapshots and lists built beforehand, release.  The hold lasts only as
      // long as these pointer swaps; nothing of it waits for Python.
      .def("switch_tables", [](Engine& e, py::list rings, py::list flow, py::list set, py::list side,
                               py::object side_ports, py::object redirects) {
        std::vector<RingEngine*> rs;
        std::vector<std::pair<bool, bool>> fs;
        for (size_t i = 0; i < rings.size(); ++i) {
          rs.push_back(rings[i].cast<RingEngine*>());
          fs.emplace_back(flow[i].cast<bool>(), set[i].cast<bool>());
        }
        std::vector<std::shared_ptr<SideTables>> st;
        for (auto o : side) st.push_back(o.is_none() ? nullptr : o.cast<std::shared_ptr<SideTables>>());
        const bool sp = !side_ports.is_none(), rd = !redirects.is_none();
        std::vector<uint32_t> spv;
        std::vector<std::pair<uint32_t, uint32_t>> rdv;
        if (sp) spv = side_ports.cast<std::vector<uint32_t>>();
        if (rd) rdv = redirects.cast<std::vector<std::pair<uint32_t, uint32_t>>>();
        std::vector<uint32_t> epochs;
        {
          py::gil_scoped_release nogil;
          e.hold();
          try {
            for (size_t i = 0; i < rs.size(); ++i) epochs.push_back(rs[i]->change_epoch(fs[i].first, fs[i].second));
            for (size_t g = 0; g < st.size(); ++g)
              if (st[g]) e.set_side_tables((uint32_t)g, st[g]);
            if (sp) e.set_side_ports(spv);
            if (rd) e.set_redirects(rdv);
          } catch (...) {
            e.release();
            throw;
          }
          e.release();
        }
        return epochs;
      }, py::arg("rings"), py::arg("flow"), py::arg("set"), py::arg("side"), py::arg("side_ports") = py::none(),
         py::arg("redirects") = py::none())
      .def("set_side_always", &Engine::set_side_always)
      .def("inject", [](Engine& e, uint32_t port, py::bytes f) {
        std::string s = f;
        e.inject(port, reinterpret_cast<const uint8_t*>(s.data()), (uint32_t)s.size());
      })
      .def("start", &Engine::start)
      .def("stop", [](Engine& e) { py::gil_scoped_release nogil; e.stop(); })
      .def("pause", [](Engine& e) { py::gil_scoped_release nogil; e.pause(); })
      .def("resume", &Engine::resume)
      .def("inject_failure", &Engine::inject_failure)
      .def_property_readonly("running", &Engine::running)
      .def("error", &Engine::error)
      .def("stats", &Engine::stats)
      .def("owner_of_frame", [](const Engine& e, py::bytes f, uint32_t port) {
        std::string s = f;
        return e.owner_of_frame(reinterpret_cast<const uint8_t*>(s.data()), (uint32_t)s.size(), port);
      })
      .def("take_punts", [](Engine& e, size_t max) {
        py::list out;
        for (auto& p : e.take_punts(max))
          out.append(py::make_tuple(py::bytes(reinterpret_cast<const char*>(p.frame.data()), p.frame.size()),
                                    (int)p.in_port, (int)p.reason));
        return out;
      }, py::arg("max") = 1024)
      .def("take_latency_us", [](Engine& e) {
        auto v = e.take_latency_us();
        return py::array_t<double>(v.size(), v.data());
      });
  m.def("owner_of_frames", [](py::array_t<uint8_t, py::array::c_style | py::array::forcecast> slots, U32Arr inmeta,
                              py::buffer ports, py::bytes rss, uint32_t n, bool v6) {
    if (slots.ndim() != 2 || slots.shape(1) != kSlotBytes || inmeta.ndim() != 1 || inmeta.shape(0) != slots.shape(0))
      throw std::invalid_argument("owner_of_frames: slots [n, 64] u8, inmeta [n] u32");
    py::buffer_info bi = ports.request();
    if ((size_t)bi.size * bi.itemsize < (size_t)kMaxPorts * sizeof(PortEntry)) throw std::invalid_argument("port table too small");
    std::string k = rss;
    if (k.size() < 20) throw std::invalid_argument("rss key too short");
    const size_t cnt = slots.shape(0);
    py::array_t<uint32_t> out(cnt);
    auto o = out.mutable_data();
    const uint8_t* sp = slots.data();
    const uint32_t* ip = inmeta.data();
    const auto* pt = static_cast<const PortEntry*>(bi.ptr);
    for (size_t i = 0; i < cnt; ++i)
      o[i] = frame_owner(sp + i * kSlotBytes, ip[i] >> 16, ip[i] & 0xFFFFu, pt, reinterpret_cast<const uint8_t*>(k.data()), n, v6);
    return out;
  }, py::arg("slots"), py::arg("inmeta"), py::arg("ports"), py::arg("rss"), py::arg("n"), py::arg("v6") = false);
  // pod side of a memif vport (tests / tools): frames in, frames out
  struct MemifEndpoint {
    std::unique_ptr<memif::Region> reg;
    memif::Producer prod;
    std::vector<memif::Consumer> cons;   // one per data plane -> pod ring
  };
  py::class_<MemifEndpoint>(m, "MemifEndpoint")
      .def(py::init([](const std::string& path) {
        auto* e = new MemifEndpoint;
        e->reg.reset(new memif::Region(path, false));
        e->prod.init(e->reg.get(), 0);
        e->cons.resize(e->reg->rx_rings());
        for (uint32_t r = 0; r < (uint32_t)e->cons.size(); ++r) e->cons[r].init(e->reg.get(), 1 + r);
        e->reg->hdr()->peer_up.store(1);
        return e;
      }))
      .def("send", [](MemifEndpoint& e, py::list frames) {
        uint32_t n = 0;
        for (auto f : frames) {
          std::string s = f.cast<py::bytes>();
          if (!e.prod.put(reinterpret_cast<const uint8_t*>(s.data()), (uint32_t)s.size())) break;
          ++n;
        }
        e.prod.commit();
        return n;
      })
      .def("recv", [](MemifEndpoint& e, uint32_t max) {
        py::list out;
        uint32_t left = max;
        for (memif::Consumer& c : e.cons) {
          const uint32_t n = std::min(c.available(), left);
          for (uint32_t i = 0; i < n; ++i) {
            uint32_t len = 0;
            const uint8_t* p = c.get(len);
            out.append(py::bytes(reinterpret_cast<const char*>(p), len));
          }
          c.release_to(c.next);
          left -= n;
        }
        return out;
      }, py::arg("max") = 4096);
  // pod-side generator / sink (trafgen.h); pods: list of (path, frames [k, stride] u8, lens [k] u32)
  m.def("cpu_share_probe", [](uint32_t threads, double seconds) {
    if (threads < 1 || threads > 1024 || !(seconds > 0.0) || seconds > 10.0)
      throw std::invalid_argument("cpu_share_probe: threads in [1, 1024], seconds in (0, 10]");
    py::gil_scoped_release nogil;
    const auto t0 = std::chrono::steady_clock::now();
    const double cpu = trafgen::cpu_share_probe(threads, seconds);
    const double wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return std::make_pair(cpu, wall);
  }, py::arg("threads"), py::arg("seconds") = 0.3,
        "threads busy-loop together: (CPU seconds granted, wall seconds); their ratio = CPUs available");
  m.def("trafgen_run", [](py::list pods, double duration_s, double warmup_s, double rate_pps, uint32_t threads,
                          uint32_t burst, uint32_t inflight) {
    std::vector<trafgen::Pod> v;
    for (auto o : pods) {
      py::tuple t = o.cast<py::tuple>();
      trafgen::Pod p;
      p.path = t[0].cast<std::string>();
      auto fr = t[1].cast<py::array_t<uint8_t, py::array::c_style | py::array::forcecast>>();
      auto ln = t[2].cast<U32Arr>();
      if (fr.ndim() != 2 || ln.ndim() != 1 || fr.shape(0) != ln.shape(0)) throw std::invalid_argument("trafgen: frames [k, stride], lens [k]");
      p.stride = (uint32_t)fr.shape(1);
      p.frames.assign(fr.data(), fr.data() + fr.size());
      p.lens.assign(ln.data(), ln.data() + ln.size());
      for (uint32_t x : p.lens) if (x > p.stride) throw std::invalid_argument("trafgen: len > stride");
      v.push_back(std::move(p));
    }
    trafgen::Config c;
    c.duration_s = duration_s; c.warmup_s = warmup_s; c.rate_pps = rate_pps; c.threads = threads; c.burst = burst;
    c.inflight = inflight;
    trafgen::Result r;
    {
      py::gil_scoped_release nogil;
      r = trafgen::run(v, c);
    }
    py::dict d;
    d["sent"] = r.sent; d["received"] = r.received; d["tx_full"] = r.tx_full; d["bad"] = r.bad;
    d["elapsed_s"] = r.elapsed_s;
    d["lat_us"] = py::array_t<double>(r.lat_us.size(), r.lat_us.data());
    d["rx_per_pod"] = r.rx_per_pod; d["tx_per_pod"] = r.tx_per_pod;
    return d;
  }, py::arg("pods"), py::arg("duration_s") = 1.0, py::arg("warmup_s") = 0.1, py::arg("rate_pps") = 0.0,
     py::arg("threads") = 1, py::arg("burst") = 32, py::arg("inflight") = 0);
  // the same generator / sink for kernel-netdev pods (trafgen_pkt.h): pods are
  // (netns path, ifname, frames [k, stride] u8, lens [k] u32)
  m.def("trafgen_run_netns", [](py::list pods, double duration_s, double warmup_s, double rate_pps, uint32_t threads,
                                uint32_t burst, bool xdp) {
    std::vector<trafgen::NetPod> v;
    for (auto o : pods) {
      py::tuple t = o.cast<py::tuple>();
      trafgen::NetPod p;
      p.netns = t[0].cast<std::string>();
      p.ifname = t[1].cast<std::string>();
      auto fr = t[2].cast<py::array_t<uint8_t, py::array::c_style | py::array::forcecast>>();
      auto ln = t[3].cast<U32Arr>();
      if (fr.ndim() != 2 || ln.ndim() != 1 || fr.shape(0) != ln.shape(0)) throw std::invalid_argument("trafgen: frames [k, stride], lens [k]");
      p.stride = (uint32_t)fr.shape(1);
      p.frames.assign(fr.data(), fr.data() + fr.size());
      p.lens.assign(ln.data(), ln.data() + ln.size());
      for (uint32_t x : p.lens) if (x > p.stride) throw std::invalid_argument("trafgen: len > stride");
      v.push_back(std::move(p));
    }
    trafgen::Config c;
    c.duration_s = duration_s; c.warmup_s = warmup_s; c.rate_pps = rate_pps; c.threads = threads; c.burst = burst;
    trafgen::Result r;
    {
      py::gil_scoped_release nogil;
      r = trafgen::run_netns(v, c, xdp);
    }
    py::dict d;
    d["sent"] = r.sent; d["received"] = r.received; d["tx_full"] = r.tx_full; d["bad"] = r.bad;
    d["elapsed_s"] = r.elapsed_s;
    d["lat_us"] = py::array_t<double>(r.lat_us.size(), r.lat_us.data());
    d["rx_per_pod"] = r.rx_per_pod; d["tx_per_pod"] = r.tx_per_pod;
    return d;
  }, py::arg("pods"), py::arg("duration_s") = 1.0, py::arg("warmup_s") = 0.1, py::arg("rate_pps") = 0.0,
     py::arg("threads") = 1, py::arg("burst") = 32, py::arg("xdp") = false);
}
