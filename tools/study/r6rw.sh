set -e
bash tools/gpu.sh r6rw py:rsoak_old:tools/router_soak.py,--seconds,60,--old-order py:rsoak_new:tools/router_soak.py,--seconds,120
