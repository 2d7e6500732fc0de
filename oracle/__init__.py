"""oracle/ — CPU restatements of RedRock's value serdes (src/rock_serdes.c). TEST INFRASTRUCTURE:
only tests/, __graft_entry__.smoke() (checker) and bench.py's cpu_baseline leg may use it."""
