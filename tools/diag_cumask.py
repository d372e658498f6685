"""Pipelined scene bench with the FCGF + matching stream (A) restricted to a CU mask (diagnostic):
python tools/diag_cumask.py <fraction of CUs for A, e.g. 0.5> [bench args].  Every k-th CU bit is kept so the mask
spreads over the XCDs."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import torch  # noqa: E402

frac = float(sys.argv[1])
orig = bench.SceneWorkload.step_pipelined


def step_pipelined(self, world):
    if not hasattr(self, "streams"):
        lib = ctypes.CDLL(os.path.join(ROOT, "tools", "vsp", "libcumask.so"))
        ncu = torch.cuda.get_device_properties(self.dev).multi_processor_count
        keep = max(1, int(round(ncu * frac)))
        bits = [0] * ncu
        step = ncu / keep
        for i in range(keep):
            bits[int(i * step)] = 1
        words = (ncu + 31) // 32
        mask = (ctypes.c_uint32 * words)()
        for i, b in enumerate(bits):
            if b:
                mask[i // 32] |= 1 << (i % 32)
        ptr = ctypes.c_void_p()
        assert lib.mvr_diag_stream_cu_mask(mask, words, ctypes.byref(ptr)) == 0
        sA = torch.cuda.ExternalStream(ptr.value, device=self.dev)
        self.streams = (sA, torch.cuda.Stream(self.dev, priority=-1), torch.cuda.Stream(self.dev, priority=-1))
        self.pending = None
        self.prepared = None
        print("stream A on %d of %d CUs" % (keep, ncu), file=sys.stderr)
    return orig(self, world)


bench.SceneWorkload.step_pipelined = step_pipelined
sys.argv = [sys.argv[0]] + sys.argv[2:]
bench.main()
