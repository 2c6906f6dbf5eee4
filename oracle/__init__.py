"""Oracle package — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import,
call, link or execute anything under oracle/.  It is the checker, never the thing
measured or shipped.
"""
