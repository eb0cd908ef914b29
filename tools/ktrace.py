import csv,sys,collections,glob
for f in sys.argv[1:]:
    print(f)
    d=collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        n=r["Kernel_Name"]
        if "hgk" not in n and "hgm" not in n: continue
        d[(n.split("(")[0], r.get("Grid_Size_X") or r.get("Grid_Size"))].append((int(r["End_Timestamp"])-int(r["Start_Timestamp"]))/1e3)
    for k,v in sorted(d.items()):
        v.sort(); print("  ", k, len(v), "median us", v[len(v)//2])
