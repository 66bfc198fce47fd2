import subprocess, sys, os
d = os.path.dirname(os.path.abspath(__file__))
for f in ("hist_temporal.py", "enc_temporal.py"):
    subprocess.run([sys.executable, os.path.join(d, f), sys.argv[1]], check=True)
