import csv,re,glob,sys
for m in sys.argv[1:]:
    g=glob.glob(f'gpurun_out/sx/{m}/*kernel_trace.csv')
    if not g: continue
    rows=list(csv.DictReader(open(g[0])))
    rows.sort(key=lambda r:int(r['Start_Timestamp']))
    seq=[(re.search(r'(k_\w+)',r['Kernel_Name']).group(1) if re.search(r'(k_\w+)',r['Kernel_Name']) else r['Kernel_Name'][:10], (int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3) for r in rows]
    sw=[round(t) for n,t in seq if n.startswith('k_sweep_')]
    print(m, sw[:8])
