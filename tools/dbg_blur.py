import sys; sys.path.insert(0,'.'); sys.path.insert(0,'tests')
import numpy as np, oracle_lib, c_orb_slam_amd as orb
from c_orb_slam_amd import synthetic
img=synthetic.sequence(0,1)[0][0]
ex=orb.ORBextractor(1200,1.2,8,20,7,max_width=1241,max_height=376)
ex(img)
e=oracle_lib.OracleExtractor(1200); e(img)
for l in range(8):
    gb,ob=ex.blurred_level(l),e.blurred(l)
    d=np.argwhere(gb!=ob)
    print("level",l,gb.shape,"ndiff",len(d))
    if len(d):
        print(" rows",np.unique(d[:,0])[:20]," cols mod 4",np.bincount(d[:,1]%4), "cols", np.unique(d[:,1])[:20])
        y,x=d[0]; print(" sample gpu",gb[y,x-2:x+6],"ora",ob[y,x-2:x+6])
        dd=(gb.astype(int)-ob.astype(int))[gb!=ob]; print(" delta hist", np.unique(dd,return_counts=True))
