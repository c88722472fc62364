// iox_xdp.cpp — AF_XDP vport of the native I/O engine (iox.h XdpPort).
//
// Raw UAPI only (linux/if_xdp.h, linux/bpf.h; no libbpf / libxdp in this image): the UMEM and its
// four rings are set up with setsockopt / mmap, and the redirect program is six BPF instructions
// loaded and attached with the bpf() syscall (BPF_PROG_LOAD, BPF_LINK_CREATE; closing the link fd
// detaches it).  The reference attaches pods to SR-IOV VF netdevs switched in NIC silicon
// (/root/reference/dpu-cni/pkgs/sriov/sriov.go:75-140); this is the software path with the least
// kernel work per frame for pods whose netdev is a veth.
#include "iox.h"

#include <errno.h>
#include <linux/bpf.h>
#include <linux/if_link.h>
#include <linux/if_xdp.h>
#include <net/if.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <cstring>
#include <stdexcept>

#ifndef AF_XDP
#define AF_XDP 44
#endif
#ifndef SOL_XDP
#define SOL_XDP 283
#endif

namespace nfdp {
namespace iox {

namespace {
uint32_t pow2_ceil(uint32_t x) {
  uint32_t p = 1;
  while (p < x) p <<= 1;
  return p;
}

long sys_bpf(int cmd, union bpf_attr* attr) { return syscall(__NR_bpf, cmd, attr, sizeof(*attr)); }

// The redirect program: r2 = ctx->rx_queue_index; r1 = xskmap; r3 = XDP_PASS (the action when the
// map has no socket for the queue); return bpf_redirect_map(r1, r2, r3).
int load_redirect_prog(int map_fd, std::string& log) {
  bpf_insn insn[6];
  std::memset(insn, 0, sizeof(insn));
  insn[0].code = BPF_LDX | BPF_MEM | BPF_W;             // r2 = *(u32 *)(r1 + offsetof(xdp_md, rx_queue_index))
  insn[0].dst_reg = BPF_REG_2;
  insn[0].src_reg = BPF_REG_1;
  insn[0].off = (int16_t)offsetof(xdp_md, rx_queue_index);
  insn[1].code = BPF_LD | BPF_DW | BPF_IMM;             // r1 = map (pseudo map fd, two slots)
  insn[1].dst_reg = BPF_REG_1;
  insn[1].src_reg = BPF_PSEUDO_MAP_FD;
  insn[1].imm = map_fd;
  insn[3].code = BPF_ALU64 | BPF_MOV | BPF_K;           // r3 = XDP_PASS
  insn[3].dst_reg = BPF_REG_3;
  insn[3].imm = XDP_PASS;
  insn[4].code = BPF_JMP | BPF_CALL;                    // r0 = bpf_redirect_map(r1, r2, r3)
  insn[4].imm = BPF_FUNC_redirect_map;
  insn[5].code = BPF_JMP | BPF_EXIT;
  static char lic[] = "GPL";
  static thread_local char buf[4096];
  buf[0] = 0;
  union bpf_attr a;
  std::memset(&a, 0, sizeof(a));
  a.prog_type = BPF_PROG_TYPE_XDP;
  a.insn_cnt = 6;
  a.insns = reinterpret_cast<uint64_t>(insn);
  a.license = reinterpret_cast<uint64_t>(lic);
  a.log_level = 1;
  a.log_size = sizeof(buf);
  a.log_buf = reinterpret_cast<uint64_t>(buf);
  a.expected_attach_type = BPF_XDP;
  std::strncpy(a.prog_name, "nfdp_xsk", sizeof(a.prog_name) - 1);
  const int fd = (int)sys_bpf(BPF_PROG_LOAD, &a);
  if (fd < 0) log = buf;
  return fd;
}
}  // namespace

XdpPort::XdpPort(const std::string& ifname, uint32_t frames, uint32_t frame_size, uint32_t queue)
    : Port(std::max<uint32_t>(frames, 64)), nframes_(pow2_ceil(std::max<uint32_t>(frames, 64))),
      fsize_(pow2_ceil(std::max<uint32_t>(frame_size, 2048))) {
  auto fail = [&](const std::string& what) {
    const int e = errno;
    close_all();   // what was set up so far
    throw std::runtime_error("iox: AF_XDP " + what + " on " + ifname + ": " + std::strerror(e));
  };
  if (fsize_ > 4096) throw std::invalid_argument("iox: AF_XDP frames are at most 4096 B");
  const unsigned ifindex = if_nametoindex(ifname.c_str());
  if (!ifindex) fail("if_nametoindex");
  fd_ = ::socket(AF_XDP, SOCK_RAW | SOCK_CLOEXEC, 0);
  if (fd_ < 0) fail("socket (needs CAP_NET_RAW)");
  // UMEM: rx frames [0, n), tx frames [n, 2n)
  umem_len_ = (size_t)2 * nframes_ * fsize_;
  void* m = mmap(nullptr, umem_len_, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_POPULATE, -1, 0);
  if (m == MAP_FAILED) { umem_ = nullptr; fail("umem mmap"); }
  umem_ = static_cast<uint8_t*>(m);
  xdp_umem_reg ur;
  std::memset(&ur, 0, sizeof(ur));
  ur.addr = reinterpret_cast<uint64_t>(umem_);
  ur.len = umem_len_;
  ur.chunk_size = fsize_;
  ur.headroom = 0;
  if (setsockopt(fd_, SOL_XDP, XDP_UMEM_REG, &ur, sizeof(ur)) != 0) fail("XDP_UMEM_REG");
  const int n = (int)nframes_;
  if (setsockopt(fd_, SOL_XDP, XDP_UMEM_FILL_RING, &n, sizeof(n)) != 0) fail("fill ring");
  if (setsockopt(fd_, SOL_XDP, XDP_UMEM_COMPLETION_RING, &n, sizeof(n)) != 0) fail("completion ring");
  if (setsockopt(fd_, SOL_XDP, XDP_RX_RING, &n, sizeof(n)) != 0) fail("rx ring");
  if (setsockopt(fd_, SOL_XDP, XDP_TX_RING, &n, sizeof(n)) != 0) fail("tx ring");
  xdp_mmap_offsets off;
  socklen_t ol = sizeof(off);
  if (getsockopt(fd_, SOL_XDP, XDP_MMAP_OFFSETS, &off, &ol) != 0) fail("XDP_MMAP_OFFSETS");
  auto map_ring = [&](Ring& r, const xdp_ring_offset& o, uint64_t pgoff, size_t desc_sz, const char* what) {
    r.map_len = o.desc + (size_t)nframes_ * desc_sz;
    void* p = mmap(nullptr, r.map_len, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_POPULATE, fd_, (off_t)pgoff);
    if (p == MAP_FAILED) { r.map = nullptr; fail(what); }
    uint8_t* b = static_cast<uint8_t*>(p);
    r.map = p;
    r.prod = reinterpret_cast<uint32_t*>(b + o.producer);
    r.cons = reinterpret_cast<uint32_t*>(b + o.consumer);
    r.flags = reinterpret_cast<uint32_t*>(b + o.flags);
    r.desc = b + o.desc;
    r.mask = nframes_ - 1;
  };
  map_ring(rx_, off.rx, XDP_PGOFF_RX_RING, sizeof(xdp_desc), "rx ring mmap");
  map_ring(tx_, off.tx, XDP_PGOFF_TX_RING, sizeof(xdp_desc), "tx ring mmap");
  map_ring(fill_, off.fr, XDP_UMEM_PGOFF_FILL_RING, sizeof(uint64_t), "fill ring mmap");
  map_ring(comp_, off.cr, XDP_UMEM_PGOFF_COMPLETION_RING, sizeof(uint64_t), "completion ring mmap");
  // every rx frame to the kernel
  uint64_t* fd = static_cast<uint64_t*>(fill_.desc);
  for (uint32_t i = 0; i < nframes_; ++i) fd[i] = (uint64_t)i * fsize_;
  __atomic_store_n(fill_.prod, nframes_, __ATOMIC_RELEASE);
  rx_addr_.assign(nframes_, 0);
  tx_free_.reserve(nframes_);
  for (uint32_t i = 0; i < nframes_; ++i) tx_free_.push_back((uint64_t)(nframes_ + i) * fsize_);
  sockaddr_xdp sa;
  std::memset(&sa, 0, sizeof(sa));
  sa.sxdp_family = AF_XDP;
  sa.sxdp_ifindex = ifindex;
  sa.sxdp_queue_id = queue;
  sa.sxdp_flags = XDP_COPY | XDP_USE_NEED_WAKEUP;
  if (bind(fd_, reinterpret_cast<sockaddr*>(&sa), sizeof(sa)) != 0) fail("bind");
  // XSKMAP[queue] = this socket, the redirect program, attached through a BPF link
  union bpf_attr a;
  std::memset(&a, 0, sizeof(a));
  a.map_type = BPF_MAP_TYPE_XSKMAP;
  a.key_size = 4;
  a.value_size = 4;
  a.max_entries = queue + 1;
  map_fd_ = (int)sys_bpf(BPF_MAP_CREATE, &a);
  if (map_fd_ < 0) fail("XSKMAP (needs CAP_BPF / CAP_NET_ADMIN)");
  const uint32_t key = queue, val = (uint32_t)fd_;
  std::memset(&a, 0, sizeof(a));
  a.map_fd = (uint32_t)map_fd_;
  a.key = reinterpret_cast<uint64_t>(&key);
  a.value = reinterpret_cast<uint64_t>(&val);
  if (sys_bpf(BPF_MAP_UPDATE_ELEM, &a) != 0) fail("XSKMAP update");
  std::string log;
  prog_fd_ = load_redirect_prog(map_fd_, log);
  if (prog_fd_ < 0) fail("program load (" + log.substr(0, 200) + ")");
  for (uint32_t mode : {(uint32_t)XDP_FLAGS_DRV_MODE, (uint32_t)XDP_FLAGS_SKB_MODE}) {
    std::memset(&a, 0, sizeof(a));
    a.link_create.prog_fd = (uint32_t)prog_fd_;
    a.link_create.target_ifindex = ifindex;
    a.link_create.attach_type = BPF_XDP;
    a.link_create.flags = mode;
    link_fd_ = (int)sys_bpf(BPF_LINK_CREATE, &a);
    if (link_fd_ >= 0) {
      native_ = mode == (uint32_t)XDP_FLAGS_DRV_MODE;
      break;
    }
  }
  if (link_fd_ < 0) fail("XDP link");
}

XdpPort::~XdpPort() { close_all(); }

void XdpPort::close_all() {
  if (link_fd_ >= 0) ::close(link_fd_);   // detaches the program
  if (prog_fd_ >= 0) ::close(prog_fd_);
  if (map_fd_ >= 0) ::close(map_fd_);
  for (Ring* r : {&rx_, &tx_, &fill_, &comp_})
    if (r->map) munmap(r->map, r->map_len);
  if (fd_ >= 0) ::close(fd_);
  if (umem_) munmap(umem_, umem_len_);
  link_fd_ = prog_fd_ = map_fd_ = fd_ = -1;
  umem_ = nullptr;
  for (Ring* r : {&rx_, &tx_, &fill_, &comp_}) r->map = nullptr;
}

uint32_t XdpPort::rx(RxRef* out, uint32_t max) {
  const uint32_t cons = *rx_.cons;
  const uint32_t avail = __atomic_load_n(rx_.prod, __ATOMIC_ACQUIRE) - cons;
  // a frame's UMEM buffer stays ours until release_to gives it back: at most nframes in hand
  const uint32_t room = nframes_ - (rx_next_ - rel_done_);
  const uint32_t n = std::min(std::min(avail, max), room);
  const xdp_desc* d = static_cast<const xdp_desc*>(rx_.desc);
  for (uint32_t i = 0; i < n; ++i) {
    const xdp_desc& x = d[(cons + i) & rx_.mask];
    const uint32_t seq = rx_next_++;
    rx_addr_[seq & (nframes_ - 1)] = x.addr;
    out[i] = RxRef{umem_ + x.addr, x.len, seq, ~0u};
  }
  if (n) __atomic_store_n(rx_.cons, cons + n, __ATOMIC_RELEASE);
  return n;
}

void XdpPort::release_to(uint32_t seq_end) {
  // frames [released .. seq_end) go back to the kernel through the fill ring
  uint32_t prod = *fill_.prod;
  uint64_t* fd = static_cast<uint64_t*>(fill_.desc);
  uint32_t k = 0;
  for (uint32_t s = rel_done_; s != seq_end; ++s, ++k) fd[(prod + k) & fill_.mask] = rx_addr_[s & (nframes_ - 1)];
  if (!k) return;
  __atomic_store_n(fill_.prod, prod + k, __ATOMIC_RELEASE);
  rel_done_ = seq_end;
  if (__atomic_load_n(fill_.flags, __ATOMIC_RELAXED) & XDP_RING_NEED_WAKEUP)
    (void)recvfrom(fd_, nullptr, 0, MSG_DONTWAIT, nullptr, nullptr);
}

void XdpPort::reclaim_tx() {
  const uint32_t cons = *comp_.cons;
  const uint32_t n = __atomic_load_n(comp_.prod, __ATOMIC_ACQUIRE) - cons;
  const uint64_t* cd = static_cast<const uint64_t*>(comp_.desc);
  for (uint32_t i = 0; i < n; ++i) tx_free_.push_back(cd[(cons + i) & comp_.mask]);
  if (n) __atomic_store_n(comp_.cons, cons + n, __ATOMIC_RELEASE);
}

void XdpPort::kick_tx() {
  // copy mode transmits inside sendto, at most a small batch per call (the kernel's TX_BATCH_SIZE,
  // 32): call it until the kernel has taken everything produced (bounded: a stuck device stops it)
  __atomic_store_n(tx_.prod, tx_prod_, __ATOMIC_RELEASE);
  for (int k = 0; k < 256 && __atomic_load_n(tx_.cons, __ATOMIC_ACQUIRE) != tx_prod_; ++k) {
    if (sendto(fd_, nullptr, 0, MSG_DONTWAIT, nullptr, 0) < 0 && errno != EAGAIN && errno != EBUSY &&
        errno != ENOBUFS)
      break;
  }
  reclaim_tx();
}

bool XdpPort::tx_locked(uint32_t, const uint8_t* a, uint32_t na, const uint8_t* b, uint32_t nb, const uint8_t* c,
                        uint32_t nc) {
  const uint32_t len = na + nb + nc;
  if (len > fsize_) return false;
  if (tx_free_.empty()) reclaim_tx();
  if (tx_free_.empty() || tx_prod_ - __atomic_load_n(tx_.cons, __ATOMIC_ACQUIRE) >= nframes_) kick_tx();
  if (tx_free_.empty()) return false;
  if (tx_prod_ - __atomic_load_n(tx_.cons, __ATOMIC_ACQUIRE) >= nframes_) return false;   // (ring full)
  const uint64_t addr = tx_free_.back();
  tx_free_.pop_back();
  uint8_t* dst = umem_ + addr;
  if (na) std::memcpy(dst, a, na);
  if (nb) std::memcpy(dst + na, b, nb);
  if (nc) std::memcpy(dst + na + nb, c, nc);
  xdp_desc& d = static_cast<xdp_desc*>(tx_.desc)[tx_prod_ & tx_.mask];
  d.addr = addr;
  d.len = len;
  d.options = 0;
  ++tx_prod_;
  return true;
}

void XdpPort::flush_locked(uint32_t) { kick_tx(); }

}  // namespace iox
}  // namespace nfdp
