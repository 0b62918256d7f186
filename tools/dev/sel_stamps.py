import numpy as np, sys
T=np.load(sys.argv[1]).astype(np.int64)
h=15*26+25
for w in range(64,72,3):
    arr=T[w,h,1]; sel=T[w,h,3]
    st=[T[w,440+k//4,k%4] for k in range(10,17)]
    print(w, 'sel', (sel-arr)/100, 'stamps', [round((s-arr)/100,2) if s>0 else None for s in st])
