"""Probe: does HIP keep a lock on pageable host memory after a copy into it returns, and is
that lock still there over a new allocation at the same address?  (the
lease-leg "illegal memory access" of rounds 4 and 5.)

The runtime (ROCclr, libamdhip64) copies a large pageable range by locking ("pinning") the
caller's pages itself (DmaBlitManager::hsaCopyStagedOrPinned -> pinHostMemory, knobs
GPU_PINNED_MIN_XFER_SIZE / GPU_PINNED_XFER_SIZE, strings in libamdhip64.so) and keeps the
pinned objects in a per-queue list for reuse, looked up by host address.  If that is so, a lock
outlives the copy, survives the caller's free(), and a later allocation at the same address
is DMA-ed through the old lock.

What this probe does (safe: it never copies into memory whose old lock it observes, and no
range it unmaps is left free for a later allocation to land in):
  (a) ten device->host copies of 8 MiB into ten live, fresh anonymous mappings, then the HSA
      pointer type of each (are the locks kept, and how many);
  (b) for each size S: a fresh anonymous mapping A, one device->host copy of S bytes into it
      through torch (HIP's pageable path), then -- with no further copy -- what the HSA runtime
      (hsa_amd_pointer_info) and HIP (hipPointerGetAttributes) report for A's address
        (1) right after the copy returned,
        (2) after munmap(A),
        (3) over a new mapping B placed at A's address (MAP_FIXED over the range just unmapped),
            which is never copied into and stays mapped until the process exits.
  HSA pointer types: 0 unknown, 1 HSA, 2 LOCKED (a host range locked for the GPU).
Writes one JSON document to stdout.
"""
import ctypes as C
import gc
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sofa-jraft_amd"))


class HsaPointerInfo(C.Structure):  # hsa_amd_pointer_info_t (hsa_ext_amd.h)
    _fields_ = [("size", C.c_uint32), ("type", C.c_int), ("agentBaseAddress", C.c_void_p),
                ("hostBaseAddress", C.c_void_p), ("sizeInBytes", C.c_size_t),
                ("userData", C.c_void_p), ("agentOwner", C.c_uint64), ("global_flags", C.c_uint32),
                ("registered", C.c_bool)]


class HipPtrAttr(C.Structure):  # hipPointerAttribute_t
    _fields_ = [("type", C.c_int), ("device", C.c_int), ("devicePointer", C.c_void_p),
                ("hostPointer", C.c_void_p), ("isManaged", C.c_int), ("allocationFlags", C.c_uint)]


def main():
    import torch
    dev = torch.device("cuda", 0)
    torch.zeros(1, device=dev)
    # the runtimes torch loaded (same SONAMEs as /opt/rocm's; NOLOAD binds the loaded copies)
    hsa = C.CDLL("libhsa-runtime64.so.1", mode=os.RTLD_NOLOAD | os.RTLD_GLOBAL)
    hip = C.CDLL("libamdhip64.so.7", mode=os.RTLD_NOLOAD | os.RTLD_GLOBAL)
    hsa.hsa_amd_pointer_info.restype = C.c_int
    hsa.hsa_amd_pointer_info.argtypes = [C.c_void_p, C.POINTER(HsaPointerInfo), C.c_void_p,
                                         C.c_void_p, C.c_void_p]
    hip.hipPointerGetAttributes.restype = C.c_int
    hip.hipGetLastError.restype = C.c_int

    def hsa_info(addr):
        i = HsaPointerInfo()
        i.size = C.sizeof(HsaPointerInfo)
        rc = hsa.hsa_amd_pointer_info(C.c_void_p(addr), C.byref(i), None, None, None)
        return {"rc": rc, "type": i.type, "host_base": hex(i.hostBaseAddress or 0),
                "agent_base": hex(i.agentBaseAddress or 0), "bytes": i.sizeInBytes}

    def hip_info(addr):
        a = HipPtrAttr()
        rc = hip.hipPointerGetAttributes(C.byref(a), C.c_void_p(addr))
        hip.hipGetLastError()
        return {"rc": rc, "type": a.type, "devicePointer": hex(a.devicePointer or 0)}

    libc = C.CDLL(None, use_errno=True)
    libc.mmap.restype = C.c_void_p
    libc.mmap.argtypes = [C.c_void_p, C.c_size_t, C.c_int, C.c_int, C.c_int, C.c_long]
    libc.munmap.argtypes = [C.c_void_p, C.c_size_t]
    PROT_RW, MAP_PRIVATE, MAP_ANON, MAP_FIXED = 0x3, 0x02, 0x20, 0x10

    def new_map(size, at=None):
        p = libc.mmap(at, size, PROT_RW, MAP_PRIVATE | MAP_ANON | (MAP_FIXED if at else 0), -1, 0)
        if p in (None, C.c_void_p(-1).value):
            raise OSError(C.get_errno(), "mmap")
        if at is not None and p != at:
            raise RuntimeError("MAP_FIXED mapping moved")
        arr = np.ctypeslib.as_array((C.c_uint8 * size).from_address(p))
        arr[::4096] = 0  # touch every page
        return p, arr

    src = torch.arange(64 << 20, dtype=torch.uint8, device=dev)  # 64 MiB device source
    torch.cuda.synchronize()
    expect = (np.arange(4096) % 256).astype(np.uint8)
    out = {"torch": torch.__version__, "hip": torch.version.hip,
           "env": {k: os.environ.get(k) for k in ("GPU_PINNED_MIN_XFER_SIZE", "GPU_PINNED_XFER_SIZE",
                                                  "GPU_STAGING_BUFFER_SIZE")},
           "cases": []}
    keep = []  # every mapping made here stays mapped (or is replaced in place) until exit
    # (a) ten live 8 MiB destinations, each copied into once
    live = [new_map(8 << 20) for _ in range(10)]
    keep += live
    for _, x in live:
        torch.from_numpy(x).copy_(src[:8 << 20])
    torch.cuda.synchronize()
    out["ten_live_8MiB_copies"] = [{"copy_ok": bool(np.array_equal(x[:4096], expect)),
                                    "hsa": hsa_info(p)} for p, x in live]
    # (b) per size: copy, then observe only
    for size in (64 << 10, 512 << 10, 1 << 20, 2 << 20, 8 << 20, 32 << 20, 48 << 20):
        pa, a = new_map(size)
        before = hsa_info(pa)
        torch.from_numpy(a).copy_(src[:size])      # D2H through HIP's pageable path
        torch.cuda.synchronize()
        ok = bool(np.array_equal(a[:4096], expect))
        after_copy = {"hsa": hsa_info(pa), "hsa_mid": hsa_info(pa + size // 2), "hip": hip_info(pa)}
        del a
        libc.munmap(C.c_void_p(pa), size)
        after_free = {"hsa": hsa_info(pa), "hip": hip_info(pa)}
        pb, b = new_map(size, at=pa)               # same address, never copied into
        keep.append((pb, b))
        over_new = {"same_address": pb == pa, "hsa": hsa_info(pb), "hsa_mid": hsa_info(pb + size // 2),
                    "hip": hip_info(pb)}
        out["cases"].append({"bytes": size, "addr": hex(pa), "copy_ok": ok, "before": before,
                             "after_copy": after_copy, "after_munmap": after_free,
                             "new_mapping_same_address": over_new})
    # (c) host->device copies from fresh mappings (the other direction), observed the same way
    out["h2d"] = []
    for size in (1 << 20, 8 << 20, 48 << 20):
        pa, a = new_map(size)
        a[:] = 7
        d = torch.empty(size, dtype=torch.uint8, device=dev)
        d.copy_(torch.from_numpy(a))
        torch.cuda.synchronize()
        out["h2d"].append({"bytes": size, "copy_ok": bool((d[:4096] == 7).all().item()),
                           "after_copy": hsa_info(pa), "after_copy_mid": hsa_info(pa + size // 2)})
        keep.append((pa, a))
        del d
    # (d) during a copy: poll the destination's HSA record from another thread while a 48 MiB
    # device->host copy runs (is the caller's range locked for the copy -- the pinned path --
    # or staged?)
    import threading
    pd, dd = new_map(48 << 20)
    keep.append((pd, dd))
    seen, stop = [], [False]

    def poll():
        while not stop[0]:
            t = hsa_info(pd + (24 << 20))["type"]
            if t and t not in seen:
                seen.append(t)
    th = threading.Thread(target=poll)
    th.start()
    for _ in range(20):
        torch.from_numpy(dd).copy_(src[:48 << 20])
    torch.cuda.synchronize()
    stop[0] = True
    th.join()
    out["during_48MiB_d2h_copies_types_seen"] = seen
    out["after_48MiB_d2h_copies"] = hsa_info(pd)
    # (e) the faulting call's own form: .cpu() of a device tensor into torch's CPU allocator,
    # then the HSA record over the result while it is alive
    t2 = torch.empty(1 << 20, dtype=torch.int16, device=dev).fill_(3)
    h2 = t2.cpu()
    out["torch_cpu_2MiB_int16"] = {"ok": bool((h2[:16] == 3).all()), "hsa": hsa_info(h2.data_ptr())}
    # (f) an explicit registration and unregistration (what libjrq's jrq_host_register does):
    # the record while registered and after hipHostUnregister
    hip.hipHostRegister.restype = C.c_int
    hip.hipHostRegister.argtypes = [C.c_void_p, C.c_size_t, C.c_uint]
    hip.hipHostUnregister.restype = C.c_int
    hip.hipHostUnregister.argtypes = [C.c_void_p]
    pr, ar = new_map(4 << 20)
    keep.append((pr, ar))
    rr = hip.hipHostRegister(C.c_void_p(pr), 4 << 20, 0)
    reg = {"hsa": hsa_info(pr), "hip": hip_info(pr)}
    ru = hip.hipHostUnregister(C.c_void_p(pr))
    out["host_register_cycle"] = {"register_rc": rr, "registered": reg, "unregister_rc": ru,
                                  "after_unregister": {"hsa": hsa_info(pr), "hip": hip_info(pr)}}
    # the instruments themselves: a hipHostMalloc'ed range (what each reports for memory HIP
    # certainly holds page-locked)
    hip.hipHostMalloc.restype = C.c_int
    hip.hipHostMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
    hp = C.c_void_p()
    rh = hip.hipHostMalloc(C.byref(hp), 1 << 20, 0)
    out["host_malloc_instrument_check"] = {"rc": rh, "hsa": hsa_info(hp.value), "hip": hip_info(hp.value)}
    # (g) r06 follow-up: sizes at and above ROCclr's pinned-transfer threshold (GPU_PINNED_MIN_XFER_SIZE,
    # 128 MiB by default as far as we know -- cases (a)-(f) all stayed below it, so they never
    # exercised the pin-in-place path the r05 bench's GiB-sized pageable uploads took).  Per size:
    # a host->device copy from a fresh mapping with a second thread polling the source's record
    # during the copy, the record after the copy, after munmap, and over a new mapping at the
    # same address (observed only, never copied into); then the same for a device->host copy.
    big_src = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
    big_src[:4096] = torch.from_numpy(expect).to(dev)
    torch.cuda.synchronize()
    out["pinned_threshold_cases"] = []

    def observe(addr, size, run):
        seen_h, seen_p, stop2 = [], [], [False]

        def poll2():
            while not stop2[0]:
                hi = hsa_info(addr + size // 2)
                if hi["type"] and hi["type"] not in seen_h:
                    seen_h.append(hi["type"])
                hp_ = hip_info(addr + size // 2)
                if hp_["type"] and hp_["type"] not in seen_p:
                    seen_p.append(hp_["type"])
        th2 = threading.Thread(target=poll2)
        th2.start()
        run()
        torch.cuda.synchronize()
        stop2[0] = True
        th2.join()
        return {"hsa_types_seen_during": seen_h, "hip_types_seen_during": seen_p}

    for size in (128 << 20, 256 << 20, 1 << 30):
        for direction in ("h2d", "d2h"):
            pa, a = new_map(size)
            if direction == "h2d":
                a[:4096] = expect
                dd2 = torch.empty(size, dtype=torch.uint8, device=dev)
                during = observe(pa, size, lambda: dd2.copy_(torch.from_numpy(a)))
                ok = bool(np.array_equal(dd2[:4096].cpu().numpy(), expect))
                del dd2
            else:
                during = observe(pa, size, lambda: torch.from_numpy(a).copy_(big_src[:size]))
                ok = bool(np.array_equal(a[:4096], expect))
            rec = {"bytes": size, "direction": direction, "copy_ok": ok, "during": during,
                   "after_copy": {"hsa": hsa_info(pa), "hsa_mid": hsa_info(pa + size // 2), "hip": hip_info(pa),
                                  "hip_mid": hip_info(pa + size // 2)}}
            del a
            libc.munmap(C.c_void_p(pa), size)
            rec["after_munmap"] = {"hsa": hsa_info(pa), "hip": hip_info(pa), "hip_mid": hip_info(pa + size // 2)}
            pb, b = new_map(size, at=pa)
            keep.append((pb, b))
            rec["new_mapping_same_address"] = {"same_address": pb == pa, "hsa": hsa_info(pb),
                                               "hip": hip_info(pb), "hip_mid": hip_info(pb + size // 2)}
            out["pinned_threshold_cases"].append(rec)
    print(json.dumps(out, indent=1))
    sys.stdout.flush()
    os._exit(0)  # leave the mappings to the kernel; no runtime teardown over the replaced ranges


if __name__ == "__main__":
    main()
