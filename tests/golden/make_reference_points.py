"""Writes tests/golden/reference_test_json_points.json: the three BLS12-381 points the reference holds in
test/test-integration/test.json (lines 2-5), as data.  The file was made by test/test-integration/json_output.go
(kyber @ 20191229, keys on G2 and signatures on G1 at the time):
    Public    = x * g2                      (96 B compressed G2: the only G2 encoding the reference holds)
    Previous  = bls.Sign(x, "Test Signature")   (48 B compressed G1, json_output.go:22)
    Signature = bls.Sign(x, Message(Previous, 1984))  with that era's 2-argument beacon.Message (json_output.go:26)
Run where /root/reference exists:  python tests/golden/make_reference_points.py"""
import json
import os

SRC = "/root/reference/test/test-integration/test.json"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_test_json_points.json")

if __name__ == "__main__":
    t = json.load(open(SRC))
    json.dump({"source": "test/test-integration/test.json:2-5 (reference), made by json_output.go:18-31",
               "round": t["Round"],
               "points": [{"name": "Public", "group": "G2", "hex": t["Public"]},
                          {"name": "Previous", "group": "G1", "hex": t["Previous"], "msg": "Test Signature"},
                          {"name": "Signature", "group": "G1", "hex": t["Signature"]}]},
              open(OUT, "w"), indent=1)
    print("wrote", OUT)
