"""Per-phase cycle counts of the LSTM step (s_memtime, workgroup 0): build lstm.hip with
-DSTZS_LSTM_PROF into a probe library (once, in this container: `python tools/probe/lstm_prof.py --build`) and run
one v0-sized recurrence (env B=64, H=256, T=80, 2 dirs; LSTM_PROF_SO = the probe library's file name).  B <= 2 takes the tagged-granule exchange (phases: sweep,
MFMA + gates, cell + publish)."""
import ctypes as C
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "styletts-zs_amd")]
import torch  # noqa: E402
from stzs import _lib as L  # noqa: E402

so = os.path.join(ROOT, "tools", "probe", os.environ.get("LSTM_PROF_SO", "liblstmprof.so"))  # A/B: another build
src = os.path.join(ROOT, "styletts-zs_amd", "csrc")
if "--build" in sys.argv or not os.path.exists(so):
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-fPIC", "-shared", "-std=c++17",
                           "-DSTZS_LSTM_PROF", "-I" + os.path.join(ROOT, "include"), "-I" + src,
                           os.path.join(src, "lstm.hip"), "-o", so])
    if "--build" in sys.argv:
        sys.exit(0)
lib = C.CDLL(so)
B, T, H = int(os.environ.get("B", 64)), int(os.environ.get("T", 80)), 256
dev = "cuda:0"
gx = torch.randn(B, T, 8 * H, device=dev) * 0.5
whh = (torch.randn(2 * 4 * H * H, device=dev) * 0.05).to(torch.bfloat16)
y = torch.zeros(B, T, 2 * H, dtype=torch.bfloat16, device=dev)
lib.stzs_lstm_workspace.restype = C.c_size_t
xchg = torch.zeros(lib.stzs_lstm_workspace(B, H, 2) // 2 + 8, dtype=torch.bfloat16, device=dev)
sync = torch.zeros(1024, dtype=torch.int64, device=dev)
a = L.LstmArgs()
a.gx, a.whhT, a.y, a.xchg, a.sync = gx.data_ptr(), whh.data_ptr(), y.data_ptr(), xchg.data_ptr(), sync.data_ptr()
a.ldg, a.bsg, a.ldy, a.bsy = 8 * H, T * 8 * H, 2 * H, T * 2 * H
a.B, a.T, a.H, a.ndir = B, T, H, 2
for it in range(3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    rc = lib.stzs_lstm(C.byref(a), C.c_void_p(torch.cuda.current_stream().cuda_stream))
    e1.record()
    torch.cuda.synchronize()
    ph = sync[257:262].cpu().tolist()
    tot = sum(ph)
    print(f"rc={rc} {e0.elapsed_time(e1)*1e3:.0f} us, per step {e0.elapsed_time(e1)*1e3/T:.2f} us; cycles/step by phase "
          f"(poll, load+sync, mfma+gates, cell+store, drain+signal): {[round(v / T) for v in ph]} total {tot / T:.0f}")
ref = os.environ.get("LSTM_REF_SO")  # compare y with another build on the same inputs
if ref:
    lib2 = C.CDLL(os.path.join(ROOT, "tools", "probe", ref))
    y0 = y.clone()
    y.zero_()
    sync.zero_()
    xchg.zero_()
    rc = lib2.stzs_lstm(C.byref(a), C.c_void_p(torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    d = (y.float() - y0.float()).abs().max().item()
    print(f"vs {ref}: rc={rc} max |dy| {d:.3e} bit-identical {torch.equal(y, y0)}")
