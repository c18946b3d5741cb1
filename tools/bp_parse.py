import sqlite3,sys
c=sqlite3.connect(sys.argv[1])
rows=list(c.execute("""select s.kernel_name, k.end-k.start from rocpd_kernel_dispatch k join rocpd_info_kernel_symbol s on k.kernel_id=s.id where s.kernel_name like '%conv_mfma%' order by k.start"""))
names=["enc.conv1","enc.conv2","blk.conv1","up.conv1","up.conv2","f0.0","f0.1","f0.2"]
nf=int(sys.argv[2]) if len(sys.argv)>2 else 4
i=0
for n in names:
    out=[]
    for fl in range(nf):
        d=[r[1] for r in rows[i:i+21]][1:]; i+=21
        d.sort(); out.append(f"{d[len(d)//2]/1e3:6.2f}")
    print(n, "  ".join(out))
