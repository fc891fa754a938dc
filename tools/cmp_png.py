import sys
sys.path[:0]=['tests','bidirectional-pathtracing_amd']
import numpy as np
from test_output_stage import read_png
a=read_png(sys.argv[1]).astype(int); b=read_png(sys.argv[2]).astype(int)
d=np.abs(a-b)
print("PNG bytes differing", int(np.count_nonzero(d)), "of", d.size, "max", int(d.max()))
