"""Mirror of the reference's `src/lib` package for the SBA / FTE path (same function
names, arguments and return values; numeric bodies on the GPU)."""
