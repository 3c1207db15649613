import csv, collections, sys, glob
d = sys.argv[1]
tot = collections.defaultdict(float); disp = set()
for f in glob.glob(f"{d}/*/*_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if (len(sys.argv) > 2 and sys.argv[2] or 'chain2aln_fast_kernel<3>') in r['Kernel_Name']:
            tot[r['Counter_Name']] += float(r['Counter_Value'])
            disp.add((f, r['Dispatch_Id']))
n = len([x for x in disp if x[0].endswith("a_counter_collection.csv")]) or 1
for k, v in sorted(tot.items()):
    print(f"{k:24s} {v/n:14.4g} per dispatch")
