"""Process footprint vs the reference pod budget (100m CPU, 200Mi; README.md:60-66): RSS, threads and
steady CPU of the CLI tracking 1 and 64 queues at 1 s polls against localhost fakes."""
import os, subprocess, sys, time, yaml
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kube_sqs_autoscaler_amd.ops import fakes, native
nat = native()
sqs, kube = fakes().FakeSqsServer(), fakes().FakeKubeServer()
sqs.start(); kube.start()
kc = "/tmp/fp_kc.yaml"
open(kc, "w").write(yaml.safe_dump({"current-context": "t", "clusters": [{"name": "c", "cluster": {"server": kube.url}}],
    "users": [{"name": "u", "user": {"token": "x"}}], "contexts": [{"name": "t", "context": {"cluster": "c", "user": "u"}}]}))
env = dict(os.environ, AWS_ACCESS_KEY_ID="a", AWS_SECRET_ACCESS_KEY="b", KUBE_CONFIG_PATH=kc)
for nq in (1, 64):
    args = [sys.executable, "-m", "kube_sqs_autoscaler_amd", "--aws-region=us-east-1", f"--sqs-endpoint={sqs.url}",
            "--poll-period=1s", "--log-level=error"]
    for i in range(nq):
        url = f"{sqs.url}/1/q{i}"
        sqs.set_attributes(url, {"ApproximateNumberOfMessages": "0", "ApproximateNumberOfMessagesDelayed": "0", "ApproximateNumberOfMessagesNotVisible": "0"})
        kube.add_deployment("ml", f"w{i}", 1)
        args += ["--queue", f"url={url},deployment=w{i},namespace=ml"]
    p = subprocess.Popen(args, cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))), env=env, stderr=subprocess.DEVNULL)
    time.sleep(6)
    st = open(f"/proc/{p.pid}/status").read()
    rss = [l for l in st.splitlines() if l.startswith(("VmRSS", "VmHWM", "Threads"))]
    t = open(f"/proc/{p.pid}/stat").read().split()
    cpu_s = (int(t[13]) + int(t[14])) / os.sysconf("SC_CLK_TCK")
    time.sleep(10)
    t2 = open(f"/proc/{p.pid}/stat").read().split()
    cpu_s2 = (int(t2[13]) + int(t2[14])) / os.sysconf("SC_CLK_TCK")
    print(nq, "queues:", rss, f"steady CPU {1000*(cpu_s2-cpu_s)/10:.1f} millicores at 1 s polls")
    p.terminate(); p.wait()
sqs.stop(); kube.stop()
