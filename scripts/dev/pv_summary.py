"""Per-kernel average times from the rocprofv3 databases written by prof_variants.sh."""
import glob, sqlite3, sys
import os
for d in sorted(glob.glob("gpurun_out/" + os.environ.get("PREFIX", "pv") + "_*")):
    if len(sys.argv) > 1 and not any(a in d for a in sys.argv[1:]):
        continue
    dbs = glob.glob(d + "/**/*.db", recursive=True)
    if not dbs:
        continue
    c = sqlite3.connect(dbs[0])
    print("==", d)
    q = "select name, count(*), avg(end-start)/1e6 from kernels group by name order by sum(end-start) desc limit 9"
    for name, cnt, ms in c.execute(q):
        print(f"  {name[:64]:64s} {cnt:4d} {ms:.3f} ms")
