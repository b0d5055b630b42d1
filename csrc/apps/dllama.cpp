#include <cstdio>
int main() { std::printf("not yet implemented\n"); return 1; }
