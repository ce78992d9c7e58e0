import csv, sys
rows=list(csv.DictReader(open(sys.argv[1])))
tot=sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:int(sys.argv[2]) if len(sys.argv)>2 else 20]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.1f} ms {float(r['TotalDurationNs'])/tot*100:5.1f}% calls {r['Calls']:>6} avg {float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:100]}")
print('total ms', tot/1e6)
