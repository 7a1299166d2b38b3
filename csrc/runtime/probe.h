// Measured device profile for the Halda-style cost partitioner (reference design
// PDF p.5 §4.1 and pp.8 §6.1-6.2: prima.cpp's Halda places layers by measured device speed).
// A pipeline stage's decode time is its weight stream through the dequant GEMV, so the speed a
// stage is weighted by is the measured GEMV weight bandwidth of its device (GB/s), with the raw
// HBM read bandwidth reported next to it.  The CPU backend measures host memcpy bandwidth.
#pragma once

namespace mp {

struct DeviceProfile {
  double hbm_read_gbps = 0;   // streaming read of a 1 GiB buffer (16 B per lane loads)
  double gemv_gbps = 0;       // Q4_K dequant GEMV, M = 1, 70B gate/up shape (weights cold)
  double speed() const { return gemv_gbps > 0 ? gemv_gbps : hbm_read_gbps; }
};

DeviceProfile probe_device(int device);   // HIP device (switches to it and back)
DeviceProfile probe_host();               // CPU backend

}  // namespace mp
