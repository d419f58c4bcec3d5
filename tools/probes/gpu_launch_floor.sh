cd "${GRAFT_REPO_ROOT}" && timeout -k 10 200 python tools/probes/launch_floor.py
