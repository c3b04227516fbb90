import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aicp_mapping_amd import synthetic as sy
pr = sy.make_pair(int(sys.argv[2]), int(sys.argv[2]), seed=int(sys.argv[3]) if len(sys.argv) > 3 else 1000)
pr.ref.tofile(sys.argv[1] + "_ref.bin"); pr.read.tofile(sys.argv[1] + "_read.bin")
