import ctypes, torch, time, os, subprocess
t0=time.time()
x = torch.arange(64, dtype=torch.float32, device="cuda")
lib = ctypes.CDLL("scripts/probe_k.so")
lib.launch.argtypes=[ctypes.c_void_p, ctypes.c_void_p]
s = torch.cuda.current_stream().cuda_stream
rc = lib.launch(ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(s))
torch.cuda.synchronize()
print("rc", rc, "ok", bool((x == 2*torch.arange(64, device="cuda", dtype=torch.float32)).all()), time.time()-t0)
print(torch.cuda.get_device_name(0), torch.cuda.get_device_properties(0))
import re
maps=open("/proc/self/maps").read()
print(sorted(set(re.findall(r"/\S*amdhip64\S*", maps))))
print("cpus", len(os.sched_getaffinity(0)), os.environ.get("OMP_NUM_THREADS"))
