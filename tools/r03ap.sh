set -e
timeout -k 10 120 python -u tools/gray_repro2.py tools/sweep_cases_r03an.json 2>&1 | grep -v Warning
