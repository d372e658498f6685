"""Pipelined scene bench with the CUs partitioned between the streams (diagnostic):
python tools/diag_cusplit.py <CUs reserved for streams A + C> <excl|bonly> [bench args].
The filter stream (B) runs on the other CUs with its persistent grids sized to them (mvr_set_cu_budget); 'excl':
streams A (FCGF + matching) and C (voxelisation) on the reserved CUs only; 'bonly': A and C unrestricted.  The
reserved CUs are spread evenly over the CU numbering (and so over the XCDs)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import torch  # noqa: E402
from lib import _native  # noqa: E402

nres = int(sys.argv[1])
mode = sys.argv[2]
orig = bench.SceneWorkload.step_pipelined


def masked_stream(lib, bits):
    words = (len(bits) + 31) // 32
    mask = (ctypes.c_uint32 * words)()
    for i, b in enumerate(bits):
        if b:
            mask[i // 32] |= 1 << (i % 32)
    ptr = ctypes.c_void_p()
    assert lib.mvr_diag_stream_cu_mask(mask, words, ctypes.byref(ptr)) == 0
    return ptr.value


def step_pipelined(self, world):
    if not hasattr(self, "streams"):
        lib = ctypes.CDLL(os.path.join(ROOT, "tools", "vsp", "libcumask.so"))
        ncu = torch.cuda.get_device_properties(self.dev).multi_processor_count
        res = [0] * ncu
        for i in range(nres):
            res[int(i * ncu / nres)] = 1
        sB = torch.cuda.ExternalStream(masked_stream(lib, [1 - b for b in res]), device=self.dev)
        prev = _native.lib().mvr_set_cu_budget(ncu - nres)
        if mode == "excl":
            sA = torch.cuda.ExternalStream(masked_stream(lib, res), device=self.dev)
            sC = torch.cuda.ExternalStream(masked_stream(lib, res), device=self.dev)
        else:
            sA, sC = torch.cuda.Stream(self.dev), torch.cuda.Stream(self.dev, priority=-1)   # bench.py's priorities
        self.streams = (sA, sB, sC)
        self.pending = None
        self.prepared = None
        print("stream B on %d of %d CUs (persistent grids sized for them, was %d); A, C %s" % (
            ncu - nres, ncu, prev, "on the other %d" % nres if mode == "excl" else "unrestricted"), file=sys.stderr)
    return orig(self, world)


bench.SceneWorkload.step_pipelined = step_pipelined
sys.argv = [sys.argv[0]] + sys.argv[3:]
bench.main()
