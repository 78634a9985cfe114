import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
g = collections.defaultdict(list)
for r in rows:
    k = r["Kernel_Name"][:70]
    gx = r.get("Grid_Size_X") or r.get("Grid_Size")
    wx = r.get("Workgroup_Size_X") or r.get("Workgroup_Size")
    lds = r.get("LDS_Block_Size") or r.get("Lds_Size")
    g[(k, gx, wx, lds)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in g.items():
    print(k, len(v), round(sorted(v)[len(v)//2], 2))
