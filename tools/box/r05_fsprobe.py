"""Per-call cost of the job-dir syscalls on the bench's temp filesystem:
mkdir vs renaming a recycled empty dir into place vs rmdir."""
import ctypes
import os
import subprocess
import tempfile
import time

base = tempfile.mkdtemp(prefix="fsprobe-")
print("tmp:", base)
print(subprocess.run(["df", "-T", base], capture_output=True, text=True).stdout)
N = 2000
libc = ctypes.CDLL(None, use_errno=True)
AT_FDCWD, NOREPLACE = -100, 1


def t(label, fn):
    t0 = time.perf_counter()
    for i in range(N):
        fn(i)
    dt = (time.perf_counter() - t0) / N * 1e6
    print(f"{label:28s} {dt:7.2f} us")


t("mkdir", lambda i: os.mkdir(f"{base}/a{i}"))
t("rename dir", lambda i: os.rename(f"{base}/a{i}", f"{base}/b{i}"))
t("renameat2 NOREPLACE dir", lambda i: libc.renameat2(AT_FDCWD, f"{base}/b{i}".encode(), AT_FDCWD,
                                                       f"{base}/c{i}".encode(), NOREPLACE))
t("rmdir", lambda i: os.rmdir(f"{base}/c{i}"))
t("makedirs exist_ok (new)", lambda i: os.makedirs(f"{base}/d{i}", exist_ok=True))
t("makedirs exist_ok (exists)", lambda i: os.makedirs(f"{base}/d{i}", exist_ok=True))
t("open O_DIRECTORY+close", lambda i: os.close(os.open(f"{base}/d{i}", os.O_RDONLY | os.O_DIRECTORY)))
os.mkdir(f"{base}/deep")
t("mkdir in subdir", lambda i: os.mkdir(f"{base}/deep/e{i}"))
