"""Host-resident packet path: pinned host slots -> SDMA -> fused kernel -> SDMA -> host.

The NAT7 role of the reference (VFIO/DPI DMA between host memory and the DPU, octep_cp_lib
soc/vfio.c) for an MI355X node whose wire side is host memory (NIC rings, AF_XDP umem, vhost
rings).  `HostPath` wraps the native engine (csrc/nfdp/pktio.hip): a producer fills slot s's
pinned `frames_in(s)` / `inmeta_in(s)` views (a NIC would DMA into them), `submit(s, n)` chains
upload, kernel and download on three streams, `results(s, n)` returns views of the processed
frames + egress metadata once the slot's download completed.  With depth >= 3, upload of batch
s+1 and download of batch s-1 overlap the kernel of batch s.
"""
from __future__ import annotations

import numpy as np

from .engine import DataPlane


class HostPath:
    def __init__(self, dp: DataPlane, capacity: int, depth: int = 3):
        if not dp.gpu:
            raise RuntimeError("HostPath needs a GPU data plane (the CPU oracle reads host memory directly)")
        self.dp = dp
        self.io = dp.nf.PacketIo(int(capacity), int(depth))
        self.capacity, self.depth = int(capacity), int(depth)
        self._n = [0] * self.depth

    def _args(self) -> dict:
        dp = self.dp
        return {"flow_ctr": dp._ptr("flow_ctr"), "port_ctr": dp._ptr("port_ctr"), "drop_ctr": dp._ptr("drop_ctr"),
                "t0": dp._ptr("t0"), "acl_wfrag": dp._ptr("acl_wfrag"), "acl_cinit": dp._ptr("acl_cinit"),
                "acl_tiles": dp._acl_tiles, "toep_frag": dp._ptr("toep_frag"), "toep_tab": dp._ptr("toep_tab"),
                "flags": 0 if dp.count_flows else 4}

    def frames_in(self, slot: int) -> np.ndarray:
        return self.io.host_in(slot)

    def inmeta_in(self, slot: int) -> np.ndarray:
        return self.io.host_inmeta(slot)

    def load(self, slot: int, frames: np.ndarray, inmeta: np.ndarray) -> int:
        """Copy a batch into slot `slot` (tests / synthetic producers; a NIC writes in place)."""
        n = len(frames)
        if n > self.capacity:
            raise ValueError("batch larger than the slot")
        self.io.wait(slot)
        self.frames_in(slot)[:n] = frames
        self.inmeta_in(slot)[:n] = np.asarray(inmeta).view(np.uint32)
        return n

    def submit(self, slot: int, n: int) -> None:
        self.dp.commit()  # pending table updates reach HBM before the batch runs
        self._n[slot] = n
        self.io.submit(slot, n, self.dp.tables_ptrs(), self._args(), self.dp.hash_mode, self.dp.acl_mode,
                       self.dp.num_cus)

    def ready(self, slot: int) -> bool:
        return self.io.ready(slot)

    def wait(self, slot: int) -> None:
        self.io.wait(slot)

    def results(self, slot: int) -> tuple[np.ndarray, np.ndarray]:
        self.io.wait(slot)
        n = self._n[slot]
        return self.io.host_out(slot)[:n], self.io.host_meta(slot)[:n]

    def timings_ms(self, slot: int) -> dict:
        h2d, kern, d2h, total = self.io.timings(slot)
        return {"h2d": h2d, "kernel": kern, "d2h": d2h, "total": total}
