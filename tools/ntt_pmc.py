import csv, collections, sys
d = sys.argv[1]
def load(name):
    rows = {}
    for r in csv.DictReader(open(f"{d}/pmc_{name}/run_counter_collection.csv")):
        if "ntt" not in r["Kernel_Name"] and "t_combine" not in r["Kernel_Name"]: continue
        k = r["Dispatch_Id"]
        rows[k] = (r["Kernel_Name"].split("(")[0].replace("void pnp::",""), int(r["Grid_Size"]), float(r["Counter_Value"]),
                   (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    return rows
F, W = load("FETCH_SIZE"), load("WRITE_SIZE")
agg = collections.defaultdict(lambda: [0, 0.0, 0.0, 0.0])
for k, (name, grid, fv, dur) in F.items():
    a = agg[(name, grid)]
    a[0] += 1; a[1] += fv * 1024 * 2; a[2] += dur
for k, (name, grid, wv, dur) in W.items():
    agg[(name, grid)][3] += wv * 1024
for (name, grid), (c, fb, dur, wb) in sorted(agg.items()):
    elems = grid * 4  # 256 lanes x 4 elements per lane (pass4), per launch
    print(f"{name:28s} grid {grid:9d} launches {c:3d}  elems {elems/2**20:6.2f}M  dur {dur/c:7.3f} ms  "
          f"fetch(x2) {fb/c/1e6:8.1f} MB  write {wb/c/1e6:8.1f} MB  alg {elems*64/1e6:8.1f} MB  "
          f"fetch/elem {fb/c/elems:5.1f} B  write/elem {wb/c/elems:5.1f} B")
