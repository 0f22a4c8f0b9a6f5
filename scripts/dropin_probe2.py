"""Per-batch timing of the drop-in call (developer probe): hbam_decode_span in 1M-record
batches from the mapped file and from a resident copy, every batch timed.
usage: python scripts/dropin_probe2.py [records] [--torch] [--pinned] [--smi] [--numa] [--steps a,b+c,...]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "hadoop-bam_amd"))
if "--torch" in sys.argv:
    import torch  # noqa: F401,E402  (before hbam: one HIP runtime)
import numpy as np  # noqa: E402
import hbam  # noqa: E402
from hbam import synth  # noqa: E402

ALL = (1 << 64) - 1


def mark(what):
    """A phase marker in both clocks a profiler trace may use (qtrace_summary.py)."""
    print(f"MARK {what} mono={time.monotonic_ns()} boot={time.clock_gettime_ns(time.CLOCK_BOOTTIME)}", flush=True)


def link_rates():
    import torch
    n = 1 << 32
    h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    d = torch.empty(n, dtype=torch.uint8, device="cuda")
    out = {}
    for name, fn in (("h2d", lambda: d.copy_(h, non_blocking=True)), ("d2h", lambda: h.copy_(d, non_blocking=True))):
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        out[name] = round(3 * n / (time.perf_counter() - t) / 1e9, 1)
    del h, d
    torch.cuda.empty_cache()
    return out


class Sampler:
    """--smi: the GPU's clock levels (pp_dpm_sclk/mclk/fclk: the starred
    level) and PCIe link speed / width from sysfs, every 20 ms while a marked
    loop runs; each loop reports the distinct values it saw, with counts."""

    FILES = ("pp_dpm_sclk", "pp_dpm_mclk", "pp_dpm_fclk", "current_link_speed", "current_link_width")

    def __init__(self):
        import glob
        import threading
        self.dev = None
        try:
            import torch
            pr = torch.cuda.get_device_properties(0)
            cand = "/sys/bus/pci/devices/%04x:%02x:%02x.0" % (getattr(pr, "pci_domain_id", 0), pr.pci_bus_id,
                                                              pr.pci_device_id)
            if os.path.exists(os.path.join(cand, "pp_dpm_sclk")):
                self.dev = cand
        except Exception:
            pass
        if self.dev is None:  # the first amdgpu device with clock files
            c = sorted(glob.glob("/sys/class/drm/card*/device/pp_dpm_sclk"))
            self.dev = os.path.dirname(c[0]) if c else None
        self.seen = {}
        self.on = False
        self.lock = threading.Lock()
        threading.Thread(target=self.run, daemon=True).start()

    def read(self):
        out = {}
        for f in self.FILES:
            try:
                txt = open(os.path.join(self.dev, f)).read()
            except OSError:
                continue
            if f.startswith("pp_dpm"):
                cur = [ln.split(":", 1)[1].replace("*", "").strip() for ln in txt.splitlines() if "*" in ln]
                out[f[7:]] = cur[0] if cur else "?"
            else:
                out[f] = txt.strip()
        return out

    def run(self):
        while True:
            if self.on and self.dev:
                v = self.read()
                with self.lock:
                    for k, x in v.items():
                        d = self.seen.setdefault(k, {})
                        d[x] = d.get(x, 0) + 1
            time.sleep(0.02)

    def start(self):
        with self.lock:
            self.seen = {}
        self.on = True

    def stop(self, label):
        self.on = False
        with self.lock:
            print(f"SMI {label} dev={self.dev} {self.seen}", flush=True)


SMI = None


def numa_summary(label):
    """--numa: where the process's large anonymous mappings (the page-locked
    batch slots and bounce buffers among them) have their pages, from
    /proc/self/numa_maps (pages per node), and the GPU's node."""
    import glob
    gnode = "?"
    for f in glob.glob("/sys/class/drm/card*/device/numa_node"):
        try:
            gnode = open(f).read().strip()
            break
        except OSError:
            pass
    rows = []
    try:
        for ln in open("/proc/self/numa_maps"):
            if "anon=" not in ln and "file=/dev/shm" not in ln:
                continue
            nodes = {k: int(v) for k, v in (t.split("=") for t in ln.split() if t[:1] == "N" and "=" in t)}
            kb = 2048 if "kernelpagesize_kB=2048" in ln else 4
            tot = sum(nodes.values()) * kb
            if tot >= 64 * 1024:
                rows.append(f"{ln.split()[0]}:{'shm' if 'file=' in ln else 'anon'}:"
                            + ",".join(f"{k}={v * kb // 1024}M" for k, v in sorted(nodes.items())))
    except OSError as e:
        rows.append(repr(e))
    print(f"NUMA {label} gpu_node={gnode} " + " ".join(rows), flush=True)


def batches(f, first, nrec):
    b = hbam.Batch()
    v, ts, n = first, [], 0
    import ctypes as C
    while True:
        t = time.perf_counter()
        rc = hbam._L.hbam_decode_span(f._h, v, ALL, nrec, C.byref(b))
        ts.append(round((time.perf_counter() - t) * 1e3, 1))
        if rc != 0 or b.n == 0:
            break
        n += b.n
        v = b.next_voff
    return n, ts


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    if "--torch" in sys.argv:  # as bench.py: torch first, its runtime initialised
        import torch
        torch.cuda.init()
        torch.empty(1, device="cuda")
    global SMI
    if "--smi" in sys.argv:
        SMI = Sampler()
        print("SMI idle", SMI.dev, SMI.read() if SMI.dev else None, flush=True)
    data, info = synth.make_bam(n, as_numpy=True)
    path = "/dev/shm/hbam_dropin_probe2.bam"
    data.tofile(path)
    del data
    try:
        steps = ["none", "gpu_load", "pinned_buffer", "run_streamed"] if "--pinned" in sys.argv else ["none", "none"]
        if "--steps" in sys.argv:
            steps = sys.argv[sys.argv.index("--steps") + 1].split(",")
        for rep, step in enumerate(steps):
            for what in step.split("+"):  # actions before this rep's measurement
                if what == "gpu_load":  # a device-resident context opened, loaded and closed
                    g = hbam.Gpu(0)
                    try:
                        g.load(np.fromfile(path, np.uint8))
                    finally:
                        g.close()
                elif what == "pinned_buffer":  # a page-locked buffer of the file, filled and freed
                    raw = np.fromfile(path, np.uint8)
                    with hbam.PinnedBuffer(raw.nbytes) as buf:
                        buf.array[:] = raw
                    del raw
                elif what == "run_streamed":  # bench.py's pinned-host leg
                    g = hbam.Gpu(0)
                    try:
                        raw = np.fromfile(path, np.uint8)
                        with hbam.PinnedBuffer(raw.nbytes) as buf:
                            buf.array[:] = raw
                            g.load(raw)
                            for _ in range(4):
                                g.run_streamed(buf.ptr, buf.nbytes, 256 << 20)
                    finally:
                        g.close()
                    del raw
                elif what == "dummy":  # a context opened and closed, nothing decoded
                    with hbam.BamFile(path=path) as fd:
                        fd.header()
                elif what == "dummy_decode":  # a context that decodes one small batch
                    with hbam.BamFile(path=path) as fd:
                        batches(fd, fd.header()["first_record_voff"], 1 << 16)
                elif what == "rates":  # torch's own pinned H2D / D2H copy rates (4 GiB), device-wide state
                    print("RATES", link_rates(), flush=True)
                elif what == "release":  # every cached device / page-locked block back to HIP
                    print("released", hbam.release_cached_memory(), flush=True)
                elif what.startswith("sleep"):  # idle seconds: a transient device state would wear off
                    time.sleep(float(what[5:] or 2))
                elif what in ("run_resident", "reload_pinned", "streamed_one_piece"):
                    g = hbam.Gpu(0)
                    try:
                        raw = np.fromfile(path, np.uint8)
                        with hbam.PinnedBuffer(raw.nbytes) as buf:
                            buf.array[:] = raw
                            g.load(raw)
                            for _ in range(4):
                                if what == "run_resident":
                                    g.run()
                                elif what == "reload_pinned":
                                    g.reload(buf.ptr, buf.nbytes, pinned=True)
                                else:
                                    g.run_streamed(buf.ptr, buf.nbytes, buf.nbytes)
                    finally:
                        g.close()
                    del raw
            print("after", step, flush=True)
            with hbam.BamFile(path=path, batch_records=1 << 20) as f:
                if "--numa" in sys.argv:
                    numa_summary(f"rep{rep}_open")
                first = f.header()["first_record_voff"]
                mark(f"mapped{rep}_begin")
                if SMI:
                    SMI.start()
                t = time.perf_counter()
                m, ts = batches(f, first, 1 << 20)
                dt = time.perf_counter() - t
                if SMI:
                    SMI.stop(f"mapped{rep}")
                mark(f"mapped{rep}_end")
                print(f"mapped rep {rep}: {m} records {dt:.3f}s {info['uncompressed'] / dt / 1e9:.1f} GB/s batches ms {ts}",
                      flush=True)
                if "--numa" in sys.argv:
                    numa_summary(f"rep{rep}_after_loop")
                t = time.perf_counter()
                f.prefetch(0, f.size)
                dtp = time.perf_counter() - t
                print(f"prefetch rep {rep}: {f.size / dtp / 1e9:.1f} GB/s host feed ({dtp * 1e3:.1f} ms)", flush=True)
                t = time.perf_counter()
                m, ts = batches(f, first, 1 << 20)
                dt = time.perf_counter() - t
                print(f"resident rep {rep}: {dt:.3f}s {info['uncompressed'] / dt / 1e9:.1f} GB/s batches ms {ts}",
                      flush=True)
    finally:
        os.unlink(path)


if __name__ == "__main__":
    main()
