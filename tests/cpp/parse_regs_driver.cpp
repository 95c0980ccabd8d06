// parse_regs_driver.cpp -- feeds RDS group registers (one unsigned 64-bit decimal per stdin line) to
// parse(bytes, chars, output, first_time) (reference src/rds_utilities.cpp:172-199, declared in
// include/rds_utilities.h) in order, with the state a fresh decoder starts from; parse prints
// PI / PTY / Program Service to stderr. Linked against the reference's own rds_utilities.o
// (oracle/_ref/parse_regs_ref, the fixture generator) or the drop-in frame layer
// (real-time-sdr_amd/host/rds_frame.cpp, the test), so both runs see identical calls.
#include <cstdint>
#include <iostream>
#include <string>

#include "rds_utilities.h"

// defined in rds_utilities.cpp:172 with external linkage; the reference's header does not declare it
void parse(const uint64_t& bytes, uint64_t& chars, uint64_t& output, bool& first_time);

int main() {
    uint64_t chars = 0, output = 0;
    bool first_time = true;
    std::string line;
    while (std::getline(std::cin, line)) {
        if (line.empty()) continue;
        const uint64_t reg = std::stoull(line);
        parse(reg, chars, output, first_time);
    }
    std::cout << chars << " " << output << " " << (first_time ? 1 : 0) << std::endl;
    return 0;
}
