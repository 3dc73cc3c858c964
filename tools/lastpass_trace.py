import csv,glob,sys
f=glob.glob(sys.argv[1]+"/**/*kernel_trace.csv",recursive=True)[0]
rows=list(csv.DictReader(open(f)))
seq=[(r["Kernel_Name"].split("(")[0].replace("void ",""),(int(r["End_Timestamp"])-int(r["Start_Timestamp"]))/1e6) for r in rows]
idx=[i for i,(n,_) in enumerate(seq) if "k_seg_init" in n]
s=idx[-1]
print(" ".join(f"{n.replace('tkz::k_seg_','').replace('<true>','').replace('<false>','')[:10]}={t:.2f}" for n,t in seq[s:s+20]))
