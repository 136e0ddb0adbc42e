import csv, collections, glob, sys
for f in sorted(glob.glob('gpurun_out/pmcc_*/run_counter_collection.csv')):
    d=collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        n=r['Kernel_Name']
        key='corr' if 'corr_nhwc' in n else 'ba' if 'ba_window_kernel' in n else 'ins' if 'pyramid_insert' in n else None
        if key: d[(key, r['Counter_Name'])].append(float(r['Counter_Value']))
    for k,v in sorted(d.items()):
        v=sorted(v); print(f.split('/')[1], k, len(v), v[len(v)//2])
