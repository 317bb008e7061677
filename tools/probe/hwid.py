import ctypes, os, sys
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libhwid.so"))
for blocks, threads in ((1, 512), (4, 512), (512, 512)):
    n = blocks * threads // 64
    buf = (ctypes.c_uint * n)()
    assert lib.run_hwid(buf, blocks, threads) == 0
    rows = []
    for i in range(min(n, 24)):
        v = buf[i]
        rows.append(f"wg{i // (threads // 64)}.w{i % (threads // 64)}: wave_id={v & 15} simd={(v >> 4) & 3} cu={(v >> 8) & 15} sh={(v >> 12) & 1} se={(v >> 13) & 7}")
    print(f"--- blocks={blocks} threads={threads}")
    print("\n".join(rows))
