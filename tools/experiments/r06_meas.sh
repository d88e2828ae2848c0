#!/bin/bash
# r06: measurement round trip on the current tree -- GPU suite + smoke, then tools/measure.sh for NS
# (kernel trace + FETCH_SIZE / WRITE_SIZE / LDS passes -> profiles/ns_traffic.json, bench line)
set -o pipefail
bash tools/measure.sh ns r06m_ns --tests
