import sys; sys.path[:0]=['tests','oracle','hadoop-bam_amd']
import numpy as np, hbam, orc
from hbam import synth
ALL=(1<<64)-1
d,_=synth.make_bam(20000)
s=orc.Stream(d); rc,want=s.decode_all()
bl=s.blocks
print('size',len(d),'blocks',len(bl), 'first coffs', [int(x) for x in bl['coff'][:6]])
for w in (1<<16, 100000, 150000, 1<<20):
    with hbam.BamFile(d, window_bytes=w) as f:
        first=f.header()['first_record_voff']
        n=0; v=first
        try:
            for b in f.iter_batches(first, ALL, 500):
                k=len(b['key'])
                ok=np.array_equal(b['voff'], want['voff'][n:n+k])
                if not ok: print('w',w,'mismatch at',n); break
                n+=k
            print('w',w,'batches ok', n, 'bytes_read', f.bytes_read())
        except Exception as e:
            print('w',w,'fail after',n,'records:',e, 'next want voff', hex(int(want['voff'][n])) if n < len(want['voff']) else None)
