"""Workgroup -> CU placement of a 2-per-CU grid (tools/probe/placement.hip): for each CU the
blockIdx values it received in the first round, summarised as the blockIdx offset between the
two workgroups that share a CU."""
import collections, ctypes, json, os
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libplacement.so"))
for blocks, lds in ((512, 72 * 1024), (1024, 72 * 1024)):
    buf = (ctypes.c_uint * (2 * blocks))()
    assert lib.run_placement(buf, blocks, lds, ctypes.c_ulonglong(200000)) == 0
    cus = collections.defaultdict(list)
    for b in range(blocks):
        hw, xcc = buf[2 * b], buf[2 * b + 1]
        key = (xcc & 15, (hw >> 13) & 7, (hw >> 12) & 1, (hw >> 8) & 15)
        cus[key].append(b)
    offs = collections.Counter()
    for v in cus.values():
        v = sorted(v)
        offs[tuple(v[i + 1] - v[i] for i in range(len(v) - 1))] += 1
    print(json.dumps({"blocks": blocks, "cus_used": len(cus), "per_cu_counts": dict(collections.Counter(len(v) for v in cus.values())),
                      "offset_patterns": {str(k): n for k, n in offs.most_common(8)},
                      "first_cus": {str(k): v for k, v in list(sorted(cus.items(), key=lambda kv: min(kv[1])))[:6]}}))
