"""Debug aid: one warm point through torj_alpha_warm (printf build)"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "torj.jl_amd"))
import torj_hip as T
r = T.alpha_warm(879645943005.1421, 0.6356810078139615, 1.123386636357144, 1.1218582593493804,
                 -0.04727651004849054, 6785.414288396569, 1.1316334434814521, mode=1, iwarm=3)
print(r)
