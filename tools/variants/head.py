# A/B baseline: the committed (HEAD) kernel sources.
import subprocess
for f in ("robust.hip", "robust_pair.hip", "robust_nets.h", "networks.inc", "robust_lds.hip", "p2p_common.h"):
    src = subprocess.run(["git", "-C", "/root/repo", "show", f"HEAD:p2pdl_amd/csrc/{f}"], check=True,
                         capture_output=True, text=True).stdout
    open(f, "w").write(src)
